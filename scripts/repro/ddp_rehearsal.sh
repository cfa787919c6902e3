#!/bin/bash
# 8-rank rehearsal of the bench.py DDP path on one GPU (gloo; ranks share the device), desync
# self-check on, and the reducer's precision probe: every bf16 bucket also reduced from an f32 copy
# of the same local gradients.  ResNet-50 b32/rank and ViT-B/16 b16/rank, the
# bucket reduction in the grad dtype (bf16) and in f32.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${DDP_OUT:-ddp}; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
P=29611
for model in "resnet50 32" "vit_b_16 16"; do
  set -- $model
  for rd in grad fp32; do
    P=$((P + 1))
    TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 TBAMD_DDP_PRECISION_PROBE=1 timeout -k 10 500 \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $P \
      bench.py --gpus 8 --model $1 --batch $2 --steps 3 --warmup 2 --reduce-dtype $rd > $O/$1_$rd.log 2>$O/$1_$rd.err
    chk $? $1_$rd
    tail -1 $O/$1_$rd.log
  done
done
echo final rc=0
