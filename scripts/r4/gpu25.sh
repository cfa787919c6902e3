#!/bin/bash
# DCGAN after the native head GEMM + tinyin wgrad: tests, steady-state census (eager and graph),
# eager vs stock
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_25; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_tinyin_wgrad.py > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed" $O/t.err | tail -2
W="timeout -k 10 500 python scripts/bench_workloads.py --workload dcgan --steps 60 --warmup 10"
for i in 1 2; do
$W --mode native > $O/dnat$i.log 2>$O/dnat$i.err; chk $? dnat$i; echo "dnat$i $(v dnat$i)"
$W --mode stock > $O/dstock$i.log 2>$O/dstock$i.err; chk $? dstock$i; echo "dstock$i $(v dstock$i)"
done
cd /tmp && export TMPDIR=/tmp
for m in eager graph; do
  g=""; [ $m = graph ] && g="--graph"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$m -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --mode native --steps 20 --warmup 10 $g > $O/tr_$m.err 2>&1; chk $? tr_$m
  python3 $R/scripts/r4/qsplit.py $(find $O/tr_$m -name '*kernel_trace.csv') --marker adamw_mt_k --last 8 --top 40 > $O/census_$m.txt; head -45 $O/census_$m.txt
  find $O/tr_$m -name '*.csv' -size +20M -delete
done
echo final rc=0
