#!/bin/bash
# staggered gemm8 correctness + speed (A/B vs unstaggered in one process), then the first pass
set -o pipefail
O=gpurun_out/r3_03; mkdir -p $O
# test failures (rc 1) are reported and the script goes on; crashes / timeouts (rc >= 124) stop it
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py tests/test_gpu_ddp.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 300 python -u scripts/gemm8_bench.py > $O/gemm8_bench.log 2>$O/gemm8_bench.err
chk $? gemm8_bench; cut -c1-330 $O/gemm8_bench.log
sed -i 's#O=gpurun_out/r3_01#O=gpurun_out/r3_03/p1#' scripts/r3/gpu01.sh
bash scripts/r3/gpu01.sh
