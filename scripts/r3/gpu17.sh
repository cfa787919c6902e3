#!/bin/bash
# 8-rank rehearsal of the driver's DDP path (torchrun env, gloo, ranks sharing the one GPU) with the
# per-step desync check; per-shape native conv fwd / dgrad / wgrad timings (ResNet-50 b256)
set -o pipefail
O=gpurun_out/r3_17; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --batch 16 --steps 3 --warmup 2 > $O/tr8.log 2>$O/tr8.err
chk $? tr8; tail -1 $O/tr8.log | cut -c1-250
timeout -k 10 400 python scripts/conv_bench.py --native-only --dgrad > $O/convs.jsonl 2>$O/convs.err; chk $? convs; tail -1 $O/convs.jsonl
