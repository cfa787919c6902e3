#!/bin/bash
# wgrad split-K partial cap A/B (32 / 16 / 8 MiB), the ResNet example vs bench.py, trajectory tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_12; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 "${@:2}" > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for i in 1 2; do
b plain$i
TBAMD_WGRAD_CAP_MB=16 b cap16_$i
TBAMD_WGRAD_CAP_MB=8 b cap8_$i
done
for c in 32 8; do
TBAMD_WGRAD_CAP_MB=$c timeout -k 10 300 python scripts/r4/wgrad_bench.py > $O/wg_$c.log 2>$O/wg_$c.err; chk $? wg_$c
done
paste -d' ' <(cut -c1-90 $O/wg_32.log) <(cut -c55-90 $O/wg_8.log)
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
