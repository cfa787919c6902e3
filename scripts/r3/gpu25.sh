#!/bin/bash
# ViT-B/16 A/B of the LDS-staged GEMM epilogue on ONE box (alternated); fp32 style-transfer and
# AdaIN native vs stock (heartbeat file: the stock first step spends minutes in MIOpen find)
set -o pipefail
O=gpurun_out/r3_25; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
for i in 1 2; do
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit$i.log 2>$O/vit$i.err; chk $? vit$i; tail -1 $O/vit$i.log | cut -c1-120; grep "'nt', 25216" $O/vit$i.err
TBAMD_GEMM8_LDS_EPI=0 TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit0$i.log 2>$O/vit0$i.err; chk $? vit0$i; tail -1 $O/vit0$i.log | cut -c1-120; grep "'nt', 25216" $O/vit0$i.err
done
for w in online adain nst; do for m in native32 stock32; do
TBAMD_TUNE_LOG=1 timeout -k 10 700 python scripts/bench_workloads.py --workload $w --mode $m --save-routes $O/routes_${w}_$m.json > $O/${w}_$m.log 2>$O/${w}_$m.err; chk $? ${w}_$m; tail -1 $O/${w}_$m.log | cut -c1-160
done; done
