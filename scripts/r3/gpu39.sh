#!/bin/bash
# tiny-channel LDS-halo weight gradient: numerics, online bf16 / fp32 re-tuned, A/B vs shipped routes
set -o pipefail
O=gpurun_out/r3_39; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_split32.py tests/test_gpu_attention.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
tune() {
TBAMD_CONV_ROUTES=none TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $1 --batch $2 --size 256 --mode $3 --steps 20 --warmup 5 --save-routes $O/routes_$1_$3.json > $O/$1_$3_tuned.log 2>$O/$1_$3_tuned.err; chk $? $1_$3_tuned; tail -1 $O/$1_$3_tuned.log | cut -c1-140; grep "miopen (\|tinyhalo" $O/$1_$3_tuned.err | cut -c1-220
}
ab() {
timeout -k 10 300 python scripts/bench_workloads.py --workload $1 --batch $2 --size 256 --mode $3 --steps 30 --warmup 5 > $O/$1_$3_old.log 2>$O/$1_$3_old.err; chk $? $1_$3_old; tail -1 $O/$1_$3_old.log | cut -c1-140
TBAMD_CONV_ROUTES=$O/routes_$1_$3.json timeout -k 10 300 python scripts/bench_workloads.py --workload $1 --batch $2 --size 256 --mode $3 --steps 30 --warmup 5 > $O/$1_$3_new.log 2>$O/$1_$3_new.err; chk $? $1_$3_new; tail -1 $O/$1_$3_new.log | cut -c1-140
}
tune online 8 native
tune online 8 native32
ab online 8 native
ab online 8 native32
