#!/bin/bash
# weight-gradient footprint, round 2: occupancy 2 combined with splits / stages / side priority
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_24; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run occ2_$i TBAMD_WGRAD_OCC=2
run occ2w2_$i TBAMD_WGRAD_OCC=2 TBAMD_WGRAD_WAVES=2
run occ2w15_$i TBAMD_WGRAD_OCC=2 TBAMD_WGRAD_WAVES=1.5
run st2_$i TBAMD_WGRAD_STAGES=2
run occ2norm_$i TBAMD_WGRAD_OCC=2 TBAMD_SIDE_PRIORITY=normal
run occ2c3_$i TBAMD_WGRAD_OCC=2 TBAMD_CONV_OCC=3
done
echo final rc=0
