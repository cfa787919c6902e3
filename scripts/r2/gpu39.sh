#!/bin/bash
# attention s_setprio A/B on ViT-B/16 (TBAMD_ATTN_PRIO=0/1 alternated on one box) + attention numerics
set -o pipefail
O=gpurun_out/r2_39; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for p in 0 1; do
    TBAMD_ATTN_PRIO=$p timeout -k 10 240 python -u bench.py --model vit_b_16 --batch 128 --steps 12 --warmup 4 > $O/vit_p${p}_$i.json 2> $O/vit_p${p}_$i.err || { tail -20 $O/vit_p${p}_$i.err; exit 1; }
    echo "prio=$p run=$i $(tail -1 $O/vit_p${p}_$i.json)"
  done
done
