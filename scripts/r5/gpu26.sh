#!/bin/bash
# new defaults (weight gradient 2 workgroups/CU incl. the BN-in-operand one, side stream at normal
# priority) vs the previous ones; streams / wgrad tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_26; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_xf.py tests/test_gpu_shared_weight.py tests/test_gpu_conv_wgrad_gemm.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
run new_$i TBAMD_X=0
run old_$i TBAMD_WGRAD_OCC=3 TBAMD_SIDE_PRIORITY=low
run occ2low_$i TBAMD_SIDE_PRIORITY=low
done
echo final rc=0
