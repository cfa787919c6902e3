#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_07; mkdir -p $O; cd $R
timeout -k 10 900 python -u scripts/tools/traj_ablation.py > $O/traj.jsonl 2> $O/traj.err; rc=$?; grep mean_x $O/traj.jsonl; exit $rc
