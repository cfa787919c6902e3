#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_09; mkdir -p $O; cd $R
VARIANTS=pure,native,nofuse N_AUTOCAST=2 SEEDS=4,5,6,7,8,9,10,11 timeout -k 10 900 python -u scripts/tools/traj_ablation.py > $O/traj8.jsonl 2> $O/traj8.err || exit $?
grep mean_x $O/traj8.jsonl
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_trajectory.py -s > $O/trajtest.log 2>&1; rc=$?; grep -E "deviation|error vs|passed|failed" $O/trajtest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/r6/gpu08.sh
