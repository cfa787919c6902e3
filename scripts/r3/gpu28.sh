#!/bin/bash
# split-bf16 fp32 conv forward / input gradient: numerics, then the fp32 style-transfer workloads
# re-tuned with it (routes saved), online also on the stock stack on the same box
set -o pipefail
O=gpurun_out/r3_28; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_split32.py tests/test_gpu_act.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
run() {
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $1 --batch $2 --size $3 --mode $4 --steps 30 --warmup 5 --save-routes $O/routes_$1_$4.json > $O/$1_$4.log 2>$O/$1_$4.err; chk $? $1_$4; tail -1 $O/$1_$4.log | cut -c1-160; grep -c "split32 (" $O/$1_$4.err
}
run online 8 256 native32
run adain 32 256 native32
run nst 1 512 native32
run online 8 256 stock32
