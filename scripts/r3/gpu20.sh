#!/bin/bash
# fused GELU-backward epilogue with batched z loads; ViT A/B (fusion on/off alternated); native
# activations; R50 + DCGAN regression check
set -o pipefail
O=gpurun_out/r3_20; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py tests/test_gpu_gelu_link.py tests/test_gpu_conv_wgrad_gemm.py tests/test_gpu_linear.py tests/test_gpu_act.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 300 python scripts/r3/gelu_bwd_bench.py > $O/gb.jsonl 2>$O/gb.err; chk $? gb; head -1 $O/gb.jsonl
for i in 1 2; do
TBAMD_GEMM_SAVE=$O/tiles_vit$i.json timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit$i.log 2>$O/vit$i.err; chk $? vit$i; tail -1 $O/vit$i.log | cut -c1-120
TBAMD_FUSE_GELU_BWD=0 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit0$i.log 2>$O/vit0$i.err; chk $? vit0$i; tail -1 $O/vit0$i.log | cut -c1-120
done
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/r50.log 2>$O/r50.err; chk $? r50; tail -1 $O/r50.log | cut -c1-120
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan > $O/dcgan.log 2>$O/dcgan.err; chk $? dcgan; tail -1 $O/dcgan.log | cut -c1-150
