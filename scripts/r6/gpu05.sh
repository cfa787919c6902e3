#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_05; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(cut -c1-150 $O/$n.json)"; }
b vit_b128 --model vit_b_16 --batch 128 --steps 20 --warmup 5
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_s128.json b vit_s128 --model vit_s_16 --batch 128 --steps 20 --warmup 5
TBAMD_TUNE_LOG=1 TBAMD_GEMM_BLAS=1 TBAMD_GEMM_TILES=$O/none.json b vit_b128_blas --model vit_b_16 --batch 128 --steps 20 --warmup 5
b vit_b128_again --model vit_b_16 --batch 128 --steps 20 --warmup 5
timeout -k 10 500 python scripts/tools/traj_ablation.py > $O/traj.jsonl 2> $O/traj.err; rc=$?; cut -c1-120 $O/traj.jsonl; exit $rc
