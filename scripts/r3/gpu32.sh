#!/bin/bash
# ResNet-50: training step on a high-priority stream (the weight-gradient side stream stays at the
# default priority, so the input-gradient chain wins dispatch) -- alternated A/B
set -o pipefail
O=gpurun_out/r3_32; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
for i in 1 2; do
TBAMD_BENCH_HIPRI=1 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/hi$i.log 2>$O/hi$i.err; chk $? hi$i; tail -1 $O/hi$i.log | cut -c1-120
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/def$i.log 2>$O/def$i.err; chk $? def$i; tail -1 $O/def$i.log | cut -c1-120
done
