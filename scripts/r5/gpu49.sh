#!/bin/bash
# after deleting the losing variants (weight-gradient 2-stage / 128-pixel paths, whole-head dQ):
# affected GPU tests + ResNet-50 and ViT-B/16 steps
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_49; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_kernels.py tests/test_gpu_xf.py tests/test_gpu_conv_wgrad_gemm.py tests/test_gpu_no_vendor_conv.py tests/test_gpu_debug.py tests/test_gpu_trajectory.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" $O/t.log | head; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/r50_$i.log 2>$O/r50_$i.err || exit 1; echo "r50_$i $(v r50_$i)"
done
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/vit128.log 2>$O/vit128.err || exit 1; echo "vit128 $(v vit128)"
timeout -k 10 300 python bench.py --model vit_b_16 > $O/vit256.log 2>$O/vit256.err || exit 1; echo "vit256 $(v vit256)"
echo final rc=0
