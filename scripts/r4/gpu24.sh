#!/bin/bash
# RGB-side 4x4/2 weight-gradient kernel (tinyin): tests, DCGAN native (routes logged) vs stock;
# then the single-stage conv occupancy A/B on the ResNet-50 step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_24; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_tinyin_wgrad.py tests/test_gpu_conv_transpose.py > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed" $O/t.err | tail -2
W="timeout -k 10 500 python scripts/bench_workloads.py --workload dcgan --steps 60 --warmup 10"
for i in 1 2; do
TBAMD_TUNE_LOG=1 $W --mode native > $O/dnat$i.log 2>$O/dnat$i.err; chk $? dnat$i; echo "dnat$i $(v dnat$i)"
$W --mode stock > $O/dstock$i.log 2>$O/dstock$i.err; chk $? dstock$i; echo "dstock$i $(v dstock$i)"
done
grep -h "(64, 3, 4, 4)" $O/dnat1.err | grep wgrad | cut -c1-220
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(v $1)"; }
for i in 1 2; do
b base$i
TBAMD_CONV_OCC=3 b focc3_$i
TBAMD_WGRAD_OCC=4 b wocc4_$i
TBAMD_WGRAD_OCC=2 b wocc2_$i
done
echo final rc=0
