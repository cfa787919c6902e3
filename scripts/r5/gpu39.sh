#!/bin/bash
# re-check of two tuning knobs at the round-5 defaults: colsum slices (TBAMD_COLSUM=min_rows,max_slices)
# and weight-gradient split waves (TBAMD_WGRAD_WAVES)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_39; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run cs32_$i TBAMD_COLSUM=32,128
run cs128_$i TBAMD_COLSUM=128,32
run ww05_$i TBAMD_WGRAD_WAVES=0.5
run ww15_$i TBAMD_WGRAD_WAVES=1.5
done
echo final rc=0
