#!/bin/bash
# A/B on one box: LN/GN affine grads into slots (TBAMD_NORM_SLOTS=1) vs copied (0); ViT-B/16 + online NST
set -o pipefail
O=gpurun_out/r2_41; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/$2.err; exit $rc; }; }
for i in 1 2; do for v in 1 0; do
  TBAMD_NORM_SLOTS=$v timeout -k 10 300 python -u bench.py --model vit_b_16 --batch 128 --steps 12 --warmup 4 > $O/vit_s${v}_$i.log 2>$O/vit_s${v}_$i.err
  chk $? vit_s${v}_$i; echo "vit slots=$v $(tail -1 $O/vit_s${v}_$i.log | cut -c70-140)"
  TBAMD_NORM_SLOTS=$v timeout -k 10 300 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --mode native --steps 20 --warmup 3 > $O/online_s${v}_$i.log 2>$O/online_s${v}_$i.err
  chk $? online_s${v}_$i; echo "online slots=$v $(tail -1 $O/online_s${v}_$i.log | cut -c70-160)"
done; done
