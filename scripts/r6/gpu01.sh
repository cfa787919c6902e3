#!/bin/bash
# round-6 opening state: carrier fix tests, headline bench, ViT bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_01; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_res_carrier.py > $O/carrier.log 2>&1; rc=$?; tail -3 $O/carrier.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.json 2> $O/vit.err || exit $?
cat $O/vit.json
TBAMD_GEMM_BLAS=0 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit_noblas.json 2> $O/vit_noblas.err || exit $?
cat $O/vit_noblas.json
