#!/bin/bash
# the restructured fp32 NST test (first-step gradient precision + trajectory band), run twice
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_32; mkdir -p $O
for i in 1 2; do
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_trajectory.py -k nst -s > $O/t$i.err 2>&1; rc=$?
echo "t$i rc=$rc"; grep -E "passed|failed|deviation|gradient error|Assert" $O/t$i.err | tail -5
[ $rc -le 1 ] || exit $rc
done
echo final rc=0
