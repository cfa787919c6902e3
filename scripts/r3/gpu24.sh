#!/bin/bash
# LDS-staged coalesced epilogue of the 8-phase GEMM: tests, NT shape A/B, ViT re-tuned A/B; then the
# fp32 style-transfer / AdaIN workloads native vs stock
set -o pipefail
O=gpurun_out/r3_24; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py tests/test_gpu_gelu_link.py tests/test_gpu_linear.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 300 python -u scripts/gemm8_bench.py > $O/g8_lds.jsonl 2>$O/g8_lds.err; chk $? g8_lds
TBAMD_GEMM8_LDS_EPI=0 timeout -k 10 300 python -u scripts/gemm8_bench.py > $O/g8_old.jsonl 2>$O/g8_old.err; chk $? g8_old
python3 -c "
import json
a=[json.loads(l) for l in open('$O/g8_lds.jsonl')]; b=[json.loads(l) for l in open('$O/g8_old.jsonl')]
for x,y in zip(a,b): print(x['shape'], 'blas', x['blas_tf'], 't16 lds', x['t16_tf'], 't16 old', y['t16_tf'])"
for i in 1 2; do
TBAMD_GEMM_SAVE=$O/tiles_vit$i.json TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit$i.log 2>$O/vit$i.err; chk $? vit$i; tail -1 $O/vit$i.log | cut -c1-120; grep "'nt', 25216" $O/vit$i.err
done
for w in online adain; do for m in native32 stock32; do
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $w --mode $m --save-routes $O/routes_${w}_$m.json > $O/${w}_$m.log 2>$O/${w}_$m.err; chk $? ${w}_$m; tail -1 $O/${w}_$m.log | cut -c1-160
done; done
