#!/bin/bash
# weight-gradient side stream restricted to a CU subset (hipExtStreamCreateWithCUMask)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_27; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run cu34_$i TBAMD_SIDE_CUS=3/4
run cu12_$i TBAMD_SIDE_CUS=1/2
run cu78_$i TBAMD_SIDE_CUS=7/8
run cu12o3_$i TBAMD_SIDE_CUS=1/2 TBAMD_WGRAD_OCC=3
done
echo final rc=0
