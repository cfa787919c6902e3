#!/bin/bash
# weight-gradient footprint, round 3: side-stream priority x occupancy x splits
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_25; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run norm_$i TBAMD_SIDE_PRIORITY=normal
run occ2norm_$i TBAMD_WGRAD_OCC=2 TBAMD_SIDE_PRIORITY=normal
run occ2normw2_$i TBAMD_WGRAD_OCC=2 TBAMD_SIDE_PRIORITY=normal TBAMD_WGRAD_WAVES=2
run occ2normw07_$i TBAMD_WGRAD_OCC=2 TBAMD_SIDE_PRIORITY=normal TBAMD_WGRAD_WAVES=0.75
done
echo final rc=0
