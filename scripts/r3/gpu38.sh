#!/bin/bash
# (1) LDS-halo tiny-channel conv: numerics + online re-tune (fp32 / bf16); (2) attention: one workgroup
# per (batch, head) for N <= 256 vs 4-wave blocks (TBAMD_ATTN_ONE_BLOCK=0), ViT-B/16 alternated
set -o pipefail
O=gpurun_out/r3_38; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_split32.py tests/test_gpu_attention.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
vit() {
TBAMD_ATTN_ONE_BLOCK=$1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit_$1_$2.log 2>$O/vit_$1_$2.err; chk $? vit_$1_$2; tail -1 $O/vit_$1_$2.log | cut -c1-110
}
vit 1 a; vit 0 a; vit 1 b; vit 0 b
tune() {
TBAMD_CONV_ROUTES=none TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $1 --batch $2 --size 256 --mode $3 --steps 20 --warmup 5 --save-routes $O/routes_$1_$3.json > $O/$1_$3_tuned.log 2>$O/$1_$3_tuned.err; chk $? $1_$3_tuned; tail -1 $O/$1_$3_tuned.log | cut -c1-140; grep "(3, 3, 9, 9)\|, 3, 9, 9)\|, 3, 3, 3)" $O/$1_$3_tuned.err | grep "fwd" | cut -c1-220
}
tune online 8 native32
tune online 8 native
tune adain 32 native
