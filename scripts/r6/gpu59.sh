#!/bin/bash
# BN apply grid bitwise-neutrality test
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_59; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_bn_grid.py > $O/t.log 2>&1; rc=$?; tail -15 $O/t.log; exit $rc
