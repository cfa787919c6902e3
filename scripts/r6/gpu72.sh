#!/bin/bash
# BN apply passes walking rows last-written-first (TBAMD_BN_REVERSE=1: memory-side-cache reuse of the
# producer's freshest lines), alternated 3x; ResNet-101 once per setting
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_72; mkdir -p $O; cd $R
for i in 1 2 3; do
for v in 0 1; do
TBAMD_BN_REVERSE=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "reverse=$v r50 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
for v in 0 1; do
TBAMD_BN_REVERSE=$v timeout -k 10 300 python bench.py --model resnet101 --steps 20 > $O/c.json 2> $O/c.err || exit $?
echo "reverse=$v r101 $(python3 -c "import json;d=json.load(open('$O/c.json'));print(d['value'])")"
done
