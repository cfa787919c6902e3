#!/bin/bash
# generalised phase-class dgrad (stride 2 any taps <= 16 / stride 3), generic native strided dgrad,
# MIOpen off by default: kernel + census tests, conv suites, headline bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_14; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.log; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_no_vendor_conv.py tests/test_gpu_kernels.py tests/test_gpu_conv_any.py tests/test_gpu_nativize.py tests/test_gpu_r4_routes.py tests/test_gpu_conv_transpose.py tests/test_gpu_convgemm.py > $O/t.log 2>&1; rc=$?; grep -n "conv kernels\|passed\|failed" $O/t.log | tail -5; chk $rc t
timeout -k 10 300 python bench.py > $O/b_1.log 2>$O/b_1.err; chk $? b_1; echo "b_1 $(v b_1)"
echo final rc=0
