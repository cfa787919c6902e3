#!/bin/bash
# re-check of the side-stream knobs after the downsample-branch byte cuts: weight-gradient occupancy,
# side-stream priority
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_52; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run occ3_$i TBAMD_WGRAD_OCC=3
run low_$i TBAMD_SIDE_PRIORITY=low
run ww15_$i TBAMD_WGRAD_WAVES=1.5
done
echo final rc=0
