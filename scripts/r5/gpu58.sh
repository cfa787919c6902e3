#!/bin/bash
# BN finalize slicing (TBAMD_COLSUM="min_rows,max_slices", default 64,64): step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_${RUN:-58}; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run def_$i TBAMD_X=0
run c32_128_$i TBAMD_COLSUM=32,128
run c16_128_$i TBAMD_COLSUM=16,128
run c32_256_$i TBAMD_COLSUM=32,256
run c16_256_$i TBAMD_COLSUM=16,256
done
echo final rc=0
