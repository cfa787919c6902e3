#!/bin/bash
# gemm8 correctness + speed, then the round-3 first pass (scripts/r3/gpu01.sh)
set -o pipefail
O=gpurun_out/r3_02; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/$2.err; exit $rc; }; }
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py > $O/gemm8_test.err 2>&1 ; chk $? gemm8_test; tail -2 $O/gemm8_test.err
timeout -k 10 300 python -u scripts/gemm8_bench.py > $O/gemm8_bench.log 2>$O/gemm8_bench.err
chk $? gemm8_bench; cat $O/gemm8_bench.log | cut -c1-400
bash scripts/r3/gpu01.sh
