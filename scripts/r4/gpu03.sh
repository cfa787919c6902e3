#!/bin/bash
# reproduce the side-stream gradient mismatch: the gpu02 order, then without the shared-weight tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_03; mkdir -p $O
run() { timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $O/t.err 2>&1; rc=$?; echo "rc=$rc $*"; grep -E "Error|assert|passed|failed" $O/t.err | tail -4 | cut -c1-300; [ $rc -le 1 ] || exit $rc; }
run tests/test_gpu_shared_weight.py tests/test_gpu_r2_correctness.py tests/test_gpu_streams.py
run tests/test_gpu_r2_correctness.py tests/test_gpu_streams.py
run tests/test_gpu_shared_weight.py tests/test_gpu_streams.py
TBAMD_HIPRI_COMPUTE=0 run tests/test_gpu_shared_weight.py tests/test_gpu_r2_correctness.py tests/test_gpu_streams.py
