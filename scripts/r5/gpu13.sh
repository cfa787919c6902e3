#!/bin/bash
# after removing the losing opt-in paths (BN fold, tiled XF forward, conv SCHED, GEMM tail split):
# the affected GPU suites, then the headline bench twice
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_13; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xf.py tests/test_gpu_conv_big.py tests/test_gpu_kernels.py tests/test_gpu_gemm8.py tests/test_gpu_gemm.py tests/test_gpu_conv1x1p.py tests/test_gpu_r4_routes.py tests/test_gpu_ddp.py tests/test_gpu_example_resnet.py > $O/t.log 2>$O/t.err; rc=$?; tail -5 $O/t.log; chk $rc t
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/b_$i.log 2>$O/b_$i.err; chk $? b_$i; echo "b_$i $(v b_$i)"
done
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/vit.log 2>$O/vit.err; chk $? vit; echo "vit $(v vit)"
echo final rc=0
