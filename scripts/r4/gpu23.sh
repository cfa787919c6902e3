#!/bin/bash
# single-stage conv occupancy re-measured on the round-4 kernels: forward 4 (default) / 3 / 2
# workgroups per CU, weight gradient 3 (default) / 4 / 2
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_23; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(v $1)"; }
for i in 1 2; do
b base$i
TBAMD_CONV_OCC=3 b focc3_$i
TBAMD_CONV_OCC=2 b focc2_$i
TBAMD_WGRAD_OCC=4 b wocc4_$i
TBAMD_WGRAD_OCC=2 b wocc2_$i
done
echo final rc=0
