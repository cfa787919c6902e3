#!/bin/bash
# BN-in-operand (XF) kernels + lazy BN in the bottleneck: tests, step A/B; streamed ImageNet
# crop kernel; the ResNet example vs bench.py; trajectory tests; ViT tile re-tune
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_13; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 "${@:2}" > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_xf.py tests/test_gpu_data.py > $O/txf.err 2>&1; chkt $? txf; grep -E "passed|failed" $O/txf.err | tail -3
for i in 1 2; do
TBAMD_BN_XF=1 b xf$i
TBAMD_BN_XF=0 b noxf$i
done
cat > $O/r50ex.yml <<YML
#include $R/examples/img_cls/resnet/resnet50_imagenet.yml
env:
  fp16: true
  n_gpu: 1
  distributed: false
dataset:
  name: synthetic:imagenet
  root: /nonexistent/imagenet
loader:
  batch_size: 256
  num_workers: 0
  pin_memory: false
  drop_last: true
YML
TBAMD_CONFIG=$O/r50ex.yml TBAMD_EXAMPLE_MAX_ITERS=50 TBAMD_EXAMPLE_TIMING=20 timeout -k 10 500 python examples/img_cls/resnet/resnet.py > $O/r50ex.log 2>$O/r50ex.err; chk $? r50ex; grep example_img_s $O/r50ex.log
b r50b
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_trajectory.py tests/test_gpu_example_resnet.py -s > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed|deviation" $O/t.err | tail -8
TBAMD_GEMM_TILES=none TBAMD_GEMM_SAVE=$O/vit_tiles.json timeout -k 10 500 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/vit_tuned.log 2>$O/vit_tuned.err; chk $? vit_tuned; tail -1 $O/vit_tuned.log | cut -c1-150
echo final rc=0
