#!/bin/bash
# retune the ViT NT/NN GEMM rows with the whole-round + tail tiles (no library candidate), then bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_04; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(cat $O/$n.json | cut -c1-200)"; }
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_b128.json b tune_b128 --model vit_b_16 --batch 128 --steps 5 --warmup 3
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_b256.json b tune_b256 --model vit_b_16 --batch 256 --steps 5 --warmup 3
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_s128.json b tune_s128 --model vit_s_16 --batch 128 --steps 5 --warmup 3
python scripts/merge_tiles.py $O/t_b128.json $O/t_b256.json $O/t_s128.json
b vit_b128 --model vit_b_16 --batch 128 --steps 20 --warmup 5
b vit_b128_2 --model vit_b_16 --batch 128 --steps 20 --warmup 5
TBAMD_GEMM_BLAS=1 TBAMD_GEMM_TILES=$O/none.json b vit_b128_blas --model vit_b_16 --batch 128 --steps 20 --warmup 5
