#!/bin/bash
# 32x32x16 big-tile conv routes: numerics, then re-time the shipped ResNet-50 routes against them
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_20; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv_big.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
TBAMD_TUNE_LOG=1 TBAMD_CONV_RETIME_M32=1 TBAMD_CONV_SAVE=$O/routes_r50.json timeout -k 10 600 python bench.py --steps 3 --warmup 2 > $O/retime.json 2> $O/retime.err || exit $?
grep "conv-retime" $O/retime.err | grep -c m32
grep "conv-retime" $O/retime.err | awk '{print $0}' | grep -- "-> big.*m32" | cut -c1-200
