#!/bin/bash
# downsample-branch carrier link (TBAMD_RES_CARRIER): numerics + failure mode, affected suites, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_50; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_res_carrier.py tests/test_gpu_kernels.py tests/test_gpu_ddp.py tests/test_gpu_xf.py tests/test_gpu_conv1x1p.py tests/test_gpu_r2_correctness.py tests/test_gpu_trajectory.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/t.log | head; tail -30 $O/t.log; exit $rc; }
for i in 1 2 3; do
timeout -k 10 300 python bench.py > $O/on_$i.log 2>$O/on_$i.err || exit 1; echo "on_$i $(v on_$i)"
TBAMD_RES_CARRIER=0 timeout -k 10 300 python bench.py > $O/off_$i.log 2>$O/off_$i.err || exit 1; echo "off_$i $(v off_$i)"
done
echo final rc=0
