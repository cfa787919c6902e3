#!/bin/bash
# the weight gradient costs 3.4 ms of the 20.7 ms step despite its side stream (skip-wgrad diagnostic:
# 14,830 vs 12,380 img/s, gpurun_out/r5_22): A/B its footprint knobs -- split count (WAVES), occupancy
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_23; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run w05_$i TBAMD_WGRAD_WAVES=0.5
run w2_$i TBAMD_WGRAD_WAVES=2
run occ2_$i TBAMD_WGRAD_OCC=2
run occ4_$i TBAMD_WGRAD_OCC=4
run cap8_$i TBAMD_WGRAD_CAP_MB=8
done
echo final rc=0
