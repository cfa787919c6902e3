#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
PROF_OUT=r6_19/vit BENCH_ARGS="--model vit_b_16 --batch 128" bash scripts/repro/profile_step.sh || exit $?
PROF_OUT=r6_19/r50 bash scripts/repro/profile_step.sh || exit $?
head -25 $R/gpurun_out/r6_19/vit/pmc_summary.txt
