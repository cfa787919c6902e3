#!/bin/bash
# split-K split32 forward for few-pixel fp32 shapes (VGG-19 b1 16²/32²): numerics, then offline fp32
# re-tuned from scratch (routes saved) vs the shipped routes on the same box
set -o pipefail
O=gpurun_out/r3_34; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_split32.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
TBAMD_CONV_ROUTES=none TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload nst --batch 1 --size 512 --mode native32 --steps 30 --warmup 5 --save-routes $O/routes_nst.json > $O/nst_tuned.log 2>$O/nst_tuned.err; chk $? nst_tuned; tail -1 $O/nst_tuned.log | cut -c1-160
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --batch 1 --size 512 --mode native32 --steps 30 --warmup 5 > $O/nst_shipped.log 2>$O/nst_shipped.err; chk $? nst_shipped; tail -1 $O/nst_shipped.log | cut -c1-160
TBAMD_CONV_ROUTES=$O/routes_nst.json timeout -k 10 300 python scripts/bench_workloads.py --workload nst --batch 1 --size 512 --mode native32 --steps 30 --warmup 5 > $O/nst_new.log 2>$O/nst_new.err; chk $? nst_new; tail -1 $O/nst_new.log | cut -c1-160
