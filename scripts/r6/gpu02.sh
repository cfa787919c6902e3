#!/bin/bash
# carrier eval/frozen fix, shared-engine census; headline + stock (nativize) + ViT benches
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_02; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_res_carrier.py tests/test_gpu_nativize.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(cat $O/$n.json)"; }
b r50 --steps 20 --warmup 5
b stock --model stock_resnet50 --steps 20 --warmup 5
b vit --model vit_b_16 --batch 128 --steps 20 --warmup 5
TBAMD_GEMM_BLAS=0 b vit_noblas --model vit_b_16 --batch 128 --steps 20 --warmup 5
