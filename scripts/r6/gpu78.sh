#!/bin/bash
# BN apply grid cap 16384 (default) vs 32768, confirmation: alternated 4x, ResNet-101 2x
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_78; mkdir -p $O; cd $R
for i in 1 2 3 4; do
for v in 16384 32768; do
TBAMD_BN_APPLY_WG=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "wg=$v r50 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
for i in 1 2; do
for v in 16384 32768; do
TBAMD_BN_APPLY_WG=$v timeout -k 10 300 python bench.py --model resnet101 --steps 20 > $O/c.json 2> $O/c.err || exit $?
echo "wg=$v r101 $(python3 -c "import json;d=json.load(open('$O/c.json'));print(d['value'])")"
done
done
