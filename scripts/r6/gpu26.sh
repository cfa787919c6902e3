#!/bin/bash
# lazy-BN test with the pinned forward route
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_26; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_xf.py > $O/xf.log 2>&1; rc=$?; tail -15 $O/xf.log; exit $rc
