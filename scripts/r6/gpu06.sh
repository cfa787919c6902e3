#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_06; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py tests/test_gpu_linear.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(cut -c1-150 $O/$n.json)"; }
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_b128.json b vit_b128_tune --model vit_b_16 --batch 128 --steps 10 --warmup 5
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_b256.json b vit_b256_tune --model vit_b_16 --batch 256 --steps 5 --warmup 3
TBAMD_TUNE_LOG=1 TBAMD_GEMM_SAVE=$O/t_s128.json b vit_s128_tune --model vit_s_16 --batch 128 --steps 5 --warmup 3
python scripts/merge_tiles.py $O/t_b128.json $O/t_b256.json $O/t_s128.json
b vit_b128 --model vit_b_16 --batch 128 --steps 20 --warmup 5
TBAMD_GEMM_BLAS=1 TBAMD_GEMM_TILES=$O/none.json b vit_b128_blas --model vit_b_16 --batch 128 --steps 20 --warmup 5
b vit_b128_2 --model vit_b_16 --batch 128 --steps 20 --warmup 5
