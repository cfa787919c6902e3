#!/bin/bash
# weight-gradient split knobs upward (cap 64 MiB, 1.5x / 2x workgroup target) vs defaults
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_34; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(v $1)"; }
for i in 1 2; do
b base$i
TBAMD_WGRAD_CAP_MB=64 b cap64_$i
TBAMD_WGRAD_WAVES=1.5 b w15_$i
TBAMD_WGRAD_CAP_MB=64 TBAMD_WGRAD_WAVES=2 b w2cap64_$i
done
echo final rc=0
