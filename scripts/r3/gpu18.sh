#!/bin/bash
# TN (weight-gradient) 8-phase GEMM: numerics tests, then timings vs the old tiles / hipBLASLt
set -o pipefail
O=gpurun_out/r3_18; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 400 python scripts/r3/gemm_tn_bench.py > $O/tn.jsonl 2>$O/tn.err; chk $? tn
python -c "
import json
for l in open('$O/tn.jsonl'):
    d=json.loads(l); print(d['shape'], 'err', d['rel_err_t16'], 't16', d['t16_best'], d['t16_ms'], d['t16_tf'], '| old', d['old_best'], d['old_ms'], d['old_tf'], '| blas', d['blas_ms'], d['blas_tf'])"
TBAMD_GEMM_SAVE=$O/tiles_vit.json timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-150; grep "'tn'" $O/vit.err
