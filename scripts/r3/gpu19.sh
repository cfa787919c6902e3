#!/bin/bash
# NN 8-phase GEMM + fused GELU backward: tests, microbench, ViT bench (nn shapes re-tuned)
set -o pipefail
O=gpurun_out/r3_19; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py tests/test_gpu_gelu_link.py tests/test_gpu_conv_wgrad_gemm.py tests/test_gpu_linear.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 300 python scripts/r3/gelu_bwd_bench.py > $O/gb.jsonl 2>$O/gb.err; chk $? gb; cat $O/gb.jsonl
TBAMD_GEMM_SAVE=$O/tiles_vit.json timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-150; grep "'nn'" $O/vit.err
TBAMD_FUSE_GELU_BWD=0 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit0.log 2>$O/vit0.err; chk $? vit0; tail -1 $O/vit0.log | cut -c1-150
