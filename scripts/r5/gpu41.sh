#!/bin/bash
# weight-gradient split-K partial cap (TBAMD_WGRAD_CAP_MB, default 32)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_41; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run cap8_$i TBAMD_WGRAD_CAP_MB=8
run cap16_$i TBAMD_WGRAD_CAP_MB=16
run cap64_$i TBAMD_WGRAD_CAP_MB=64
done
echo final rc=0
