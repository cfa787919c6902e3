#!/bin/bash
# gemm8 (B0 kept in registers): tests + bench; plain ResNet-50 kernel trace (vs the --ddp one of r3_03)
set -o pipefail
O=gpurun_out/r3_06; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py > $O/t.err 2>&1 ; chk $? t; tail -1 $O/t.err
timeout -k 10 300 python -u scripts/gemm8_bench.py > $O/gemm8_bench.log 2>$O/gemm8_bench.err
chk $? gemm8_bench; python3 -c "
import json
for l in open('$O/gemm8_bench.log'):
    d=json.loads(l); print(d['shape'], 'blas', d['blas_tf'], 't16', d['t16_tf'], 't16ns', d['t16ns_tf'], 't0', d['t0_tf'], 't1', d['t1_tf'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r50 -- python bench.py --steps 4 --warmup 3 > $O/prof.log 2>&1
chk $? prof
