#!/bin/bash
# conv weight-gradient split-K partial cap (TBAMD_WGRAD_CAP_MB 32 default / 16 / 48) on the final BN tree, alternated 3x
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_81; mkdir -p $O; cd $R
for i in 1 2 3; do
for v in 32 16 48; do
TBAMD_WGRAD_CAP_MB=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "cap=$v r50 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
for v in 32 16 48; do
TBAMD_WGRAD_CAP_MB=$v timeout -k 10 300 python bench.py --model resnet101 --steps 20 > $O/c.json 2> $O/c.err || exit $?
echo "cap=$v r101 $(python3 -c "import json;d=json.load(open('$O/c.json'));print(d['value'])")"
done
