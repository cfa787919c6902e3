#!/bin/bash
# BN applies: plain reverse (1) vs interleaved 8-segment reverse (2, matches the producer conv XCD ranges)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_75; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bn_grid.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3 4; do
for v in 1 2; do
TBAMD_BN_REVERSE=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "reverse=$v r50 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
for i in 1 2; do
for v in 1 2; do
TBAMD_BN_REVERSE=$v timeout -k 10 300 python bench.py --model resnet101 --steps 20 > $O/c.json 2> $O/c.err || exit $?
echo "reverse=$v r101 $(python3 -c "import json;d=json.load(open('$O/c.json'));print(d['value'])")"
done
done
