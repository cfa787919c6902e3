#!/bin/bash
# fp32 RGB-head weight gradients (split-bf16 halo-tile runs): numerics, online / AdaIN fp32 re-tuned
set -o pipefail
O=gpurun_out/r3_29; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wgrad_split32.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
run() {
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $1 --batch $2 --size $3 --mode native32 --steps 30 --warmup 5 --save-routes $O/routes_$1.json > $O/$1.log 2>$O/$1.err; chk $? $1; tail -1 $O/$1.log | cut -c1-160; grep "narrow32\|miopen)" $O/$1.err | cut -c1-200 || true
}
run online 8 256
run adain 32 256
