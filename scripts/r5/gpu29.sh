#!/bin/bash
# 128-pixel k-tiles for the weight gradient (TBAMD_WGRAD_BK=128): numerics under that env, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_29; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
TBAMD_WGRAD_BK=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_xf.py tests/test_gpu_conv_wgrad_gemm.py tests/test_gpu_no_vendor_conv.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
run base_$i TBAMD_X=0
run bk128_$i TBAMD_WGRAD_BK=128
done
echo final rc=0
