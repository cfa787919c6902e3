#!/bin/bash
# DDP path after the downsample-branch links (carrier + lazy affine): 4-rank gloo rehearsal on one GPU,
# desync self-check on, ResNet-50 b32/rank
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_55; mkdir -p $O
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 500 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29655 \
  bench.py --gpus 4 --model resnet50 --batch 32 --steps 3 --warmup 2 > $O/r50.log 2>$O/r50.err || { echo "ddp failed"; tail -30 $O/r50.err; exit 1; }
tail -1 $O/r50.log | cut -c1-300
grep -i "desync\|check" $O/r50.err | tail -3
echo final rc=0
