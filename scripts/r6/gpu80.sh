#!/bin/bash
# BN apply minimum row passes per workgroup (TBAMD_BN_APPLY_MINPASS 2 default / 1 / 4) at the 32768 cap, alternated 3x
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_80; mkdir -p $O; cd $R
for i in 1 2 3; do
for v in 2 1 4; do
TBAMD_BN_APPLY_MINPASS=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "minpass=$v r50 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
for v in 2 1 4; do
TBAMD_BN_APPLY_MINPASS=$v timeout -k 10 300 python bench.py --model resnet101 --steps 20 > $O/c.json 2> $O/c.err || exit $?
echo "minpass=$v r101 $(python3 -c "import json;d=json.load(open('$O/c.json'));print(d['value'])")"
done
