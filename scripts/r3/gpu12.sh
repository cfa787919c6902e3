#!/bin/bash
set -o pipefail
O=gpurun_out/r3_12; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_any.py tests/test_gpu_streams.py tests/test_gpu_gram.py tests/test_gpu_trajectory.py tests/test_gpu_ddp.py tests/test_gpu_convgemm.py tests/test_gpu_linear.py tests/test_gpu_r2_correctness.py > $O/t.err 2>&1 ; chk $? t; tail -3 $O/t.err
PYTHONPATH=. timeout -k 10 300 python scripts/r3/f32_conv_bench.py > $O/f32.jsonl 2> $O/f32.err; chk $? f32; cat $O/f32.jsonl
