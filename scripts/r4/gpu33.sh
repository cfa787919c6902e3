#!/bin/bash
# the driver's multi-rank bench path rehearsed on one GPU: 2 ranks (gloo, both on GPU 0) through
# torch.distributed.run with the gradient desync check, ResNet-50 (BN-in-operand default on) and ViT
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_33; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
export TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 6 --warmup 4 --batch 64 > $O/r50_2r.log 2>$O/r50_2r.err; chk $? r50_2r; tail -1 $O/r50_2r.log | cut -c1-300; grep -i "desync\|identical\|check" $O/r50_2r.err | tail -3
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --model vit_b_16 --steps 4 --warmup 3 --batch 32 > $O/vit_2r.log 2>$O/vit_2r.err; chk $? vit_2r; tail -1 $O/vit_2r.log | cut -c1-300; grep -i "desync\|identical\|check" $O/vit_2r.err | tail -3
echo final rc=0
