#!/bin/bash
# GraphedStep after the pinned staging ring: graph tests, DCGAN eager vs graph alternated, LeNet/VAE graph
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_28; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_graph_step.py > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed" $O/t.err | tail -2
W="timeout -k 10 500 python scripts/bench_workloads.py --workload dcgan --steps 100 --warmup 10"
for i in 1 2; do
$W --mode native > $O/eager$i.log 2>$O/eager$i.err; chk $? eager$i; echo "eager$i $(v eager$i)"
$W --mode native --graph > $O/graph$i.log 2>$O/graph$i.err; chk $? graph$i; echo "graph$i $(v graph$i)"
done
for w in lenet vae; do
timeout -k 10 300 python scripts/bench_workloads.py --workload $w --mode native --graph --steps 200 --warmup 10 --batch 256 > $O/$w.log 2>$O/$w.err; chk $? $w; echo "$w $(v $w)"
done
echo final rc=0
