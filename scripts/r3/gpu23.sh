#!/bin/bash
# DCGAN: native with the frozen-D G step, eager and hipGraph-replayed, vs stock (same box)
set -o pipefail
O=gpurun_out/r3_23; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
for i in 1 2; do
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 60 --warmup 10 > $O/nat$i.log 2>$O/nat$i.err; chk $? nat$i; tail -1 $O/nat$i.log | cut -c1-140
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --graph --steps 60 --warmup 10 > $O/natg$i.log 2>$O/natg$i.err; chk $? natg$i; tail -1 $O/natg$i.log | cut -c1-140
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode stock --steps 60 --warmup 10 > $O/stock$i.log 2>$O/stock$i.err; chk $? stock$i; tail -1 $O/stock$i.log | cut -c1-140
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gelu_link.py tests/test_gpu_gemm8.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 300 python scripts/r3/gelu_bwd_bench.py > $O/gb.jsonl 2>$O/gb.err; chk $? gb; head -1 $O/gb.jsonl
for i in 1 2; do
TBAMD_FUSE_GELU_BWD=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vitf$i.log 2>$O/vitf$i.err; chk $? vitf$i; tail -1 $O/vitf$i.log | cut -c1-120
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vitu$i.log 2>$O/vitu$i.err; chk $? vitu$i; tail -1 $O/vitu$i.log | cut -c1-120
done
