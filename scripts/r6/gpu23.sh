#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_23; mkdir -p $O; cd $R
TBAMD_TUNE_LOG=1 TBAMD_CONV_RETIME=big64x256,big64x256m32 TBAMD_CONV_SAVE=$O/routes.json timeout -k 10 600 python bench.py --steps 3 --warmup 2 > $O/retime.json 2> $O/retime.err || exit $?
grep -c "conv-retime" $O/retime.err
grep "conv-retime" $O/retime.err | cut -c1-220
