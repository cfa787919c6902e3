#!/bin/bash
# style-transfer workloads at the reference configs and precision (fp32): online b8 @256, AdaIN b32
# @256, offline VGG-19 b1 @512 -- native vs stock; heartbeat file for the stock MIOpen find
set -o pipefail
O=gpurun_out/r3_26; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
run() {  # workload batch size
for m in native32 stock32; do
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $1 --batch $2 --size $3 --mode $m --steps 30 --warmup 5 --save-routes $O/routes_$1_$m.json > $O/$1_$m.log 2>$O/$1_$m.err; chk $? $1_$m; tail -1 $O/$1_$m.log | cut -c1-160
done
}
run online 8 256
run adain 32 256
run nst 1 512
