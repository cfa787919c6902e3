#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_07; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_gpu_conv_big.py -k heuristic tests/test_gpu_linear.py tests/test_gpu_gram.py tests/test_gpu_convgemm.py tests/test_gpu_f32_exact.py > $O/t.err 2>&1; echo "t rc=$?"; grep -E "deviation|^exact|passed|failed|FAILED" $O/t.err | tail -12
VB="bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8"
for i in 1 2; do
timeout -k 10 300 python $VB > $O/vit_$i.log 2>$O/vit_$i.err; chk $? vit_$i; echo "vit_$i $(v vit_$i)"
TBAMD_GEMM_BLAS=0 timeout -k 10 300 python $VB > $O/vitnat_$i.log 2>$O/vitnat_$i.err; chk $? vitnat_$i; echo "vitnat_$i $(v vitnat_$i)"
done
bash scripts/repro/ddp_rehearsal.sh 2>&1 | tail -12
echo final rc=0
