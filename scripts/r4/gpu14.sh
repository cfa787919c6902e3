#!/bin/bash
# XF (BN + ReLU in the consumer conv's operand staging) after the LDS-coefficient fix and the
# backward without re-materialisation: tests, step A/B, queue-split traces XF on / off
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_14; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 "${@:2}" > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_xf.py tests/test_gpu_data.py tests/test_gpu_debug.py tests/test_gpu_attention.py > $O/txf.err 2>&1; chkt $? txf; grep -E "passed|failed" $O/txf.err | tail -3
for i in 1 2; do
TBAMD_BN_XF=1 b xf$i
TBAMD_BN_XF=0 b noxf$i
done
for v in 1 0; do
TBAMD_BN_XF=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_xf$v -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr_xf$v.err 2>&1; chk $? tr_xf$v
python3 $R/scripts/r4/qsplit.py $(find $O/tr_xf$v -name '*kernel_trace.csv') --top 45 > $O/qsplit_xf$v.txt; head -4 $O/qsplit_xf$v.txt
done
b vit --model vit_b_16 --batch 128
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_vit -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 3 --warmup 3 > $O/tr_vit.err 2>&1; chk $? tr_vit
python3 $R/scripts/r4/qsplit.py $(find $O/tr_vit -name '*kernel_trace.csv') --top 30 > $O/qsplit_vit.txt; head -20 $O/qsplit_vit.txt
echo final rc=0
