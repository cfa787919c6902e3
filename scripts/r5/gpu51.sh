#!/bin/bash
# lazy affine downsample output (TBAMD_LAZY_DS): numerics, affected suites, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_51; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 900 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/t.log | head; tail -30 $O/t.log; exit $rc; }
for i in 1 2 3; do
timeout -k 10 300 python bench.py > $O/on_$i.log 2>$O/on_$i.err || exit 1; echo "on_$i $(v on_$i)"
TBAMD_LAZY_DS=0 timeout -k 10 300 python bench.py > $O/off_$i.log 2>$O/off_$i.err || exit 1; echo "off_$i $(v off_$i)"
done
echo final rc=0
