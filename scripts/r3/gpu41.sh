#!/bin/bash
# closing DCGAN native vs stock (alternated, same box) on the final round-3 tree
set -o pipefail
O=gpurun_out/r3_41; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
for i in 1 2; do
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 60 --warmup 10 > $O/nat$i.log 2>$O/nat$i.err; chk $? nat$i; tail -1 $O/nat$i.log | cut -c1-140
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode stock --steps 60 --warmup 10 > $O/stock$i.log 2>$O/stock$i.err; chk $? stock$i; tail -1 $O/stock$i.log | cut -c1-140
done
