#!/bin/bash
# DCGAN-128 G+D step: eager vs one replayed hipGraph (utils.GraphedStep over both optimizers),
# alternated with stock; the fp32 NST trajectory test; ViT GEMM tiles shipped vs re-tuned
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_19; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
W="timeout -k 10 500 python scripts/bench_workloads.py --workload dcgan --steps 100 --warmup 10"
for i in 1 2; do
$W --mode native > $O/eager$i.log 2>$O/eager$i.err; chk $? eager$i; echo "eager$i $(v eager$i)"
$W --mode native --graph > $O/graph$i.log 2>$O/graph$i.err; chk $? graph$i; echo "graph$i $(v graph$i)"
$W --mode stock > $O/stock$i.log 2>$O/stock$i.err; chk $? stock$i; echo "stock$i $(v stock$i)"
done
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_trajectory.py -k nst -s > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed|deviation" $O/t.err | tail -3
for i in 1 2; do
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/vship$i.log 2>$O/vship$i.err; chk $? vship$i; echo "vship$i $(v vship$i)"
done
echo final rc=0
