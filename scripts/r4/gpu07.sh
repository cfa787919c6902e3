#!/bin/bash
# gemm8 tail split-K: numerics, per-shape A/B vs hipBLASLt, ViT bench with and without the library
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_07; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
# test steps: a failing test (rc 1) is reported and the script goes on; a crash / timeout stops it
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_gemm8_sk.py > $O/sk.err 2>&1; chkt $? sk; grep -E "passed|failed" $O/sk.err | tail -2
timeout -k 10 300 python scripts/r4/vit_gemm_bench.py > $O/vg.log 2>$O/vg.err; chk $? vg; cat $O/vg.log
for i in 1 2; do
timeout -k 10 400 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit$i.log 2>$O/vit$i.err; chk $? vit$i; tail -1 $O/vit$i.log | cut -c1-150
TBAMD_GEMM_BLAS=0 timeout -k 10 400 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vitn$i.log 2>$O/vitn$i.err; chk $? vitn$i; tail -1 $O/vitn$i.log | cut -c1-150
done
cd /tmp && export TMPDIR=/tmp
TBAMD_GEMM_BLAS=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_vit -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 3 --warmup 3 > $O/tr_vit.err 2>&1; chk $? tr_vit
python3 $R/scripts/r4/qsplit.py $(find $O/tr_vit -name '*kernel_trace.csv') --top 24 > $O/vit_qsplit.txt; head -40 $O/vit_qsplit.txt
