#!/bin/bash
# multi-rank rehearsal of bench.py's DDP path on one GPU (ranks share cuda:0 over gloo, gradient
# desync self-check on) + the 1-rank RCCL DDP bench, on the current tree
set -o pipefail
O=gpurun_out/r2_40; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 $O/$2.err; exit $rc; }; }
[ "$SKIP_PYTEST" = 1 ] || { timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_layernorm.py > $O/pytest.err 2>&1 ; chk $? pytest; tail -1 $O/pytest.err; }
timeout -k 10 300 python -u bench.py --model vit_b_16 --batch 128 --steps 12 --warmup 4 > $O/vit.log 2>$O/vit.err
chk $? vit; tail -1 $O/vit.log | cut -c1-200
timeout -k 10 300 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --mode native --steps 10 --warmup 3 > $O/online.log 2>$O/online.err
chk $? online; tail -1 $O/online.log | cut -c1-200
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --batch 32 --steps 3 --warmup 2 > $O/r50_ddp2.log 2>$O/r50_ddp2.err
chk $? r50_ddp2; tail -1 $O/r50_ddp2.log | cut -c1-200
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 4 --batch 16 --steps 3 --warmup 2 > $O/r50_ddp4.log 2>$O/r50_ddp4.err
chk $? r50_ddp4; tail -1 $O/r50_ddp4.log | cut -c1-200
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29615 bench.py --gpus 2 --model vit_b_16 --batch 16 --steps 3 --warmup 2 > $O/vit_ddp2.log 2>$O/vit_ddp2.err
chk $? vit_ddp2; tail -1 $O/vit_ddp2.log | cut -c1-200
timeout -k 10 300 python bench.py --ddp --steps 20 --warmup 5 > $O/r50_ddp1_rccl.log 2>$O/r50_ddp1_rccl.err
chk $? r50_ddp1_rccl; tail -1 $O/r50_ddp1_rccl.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r50.log 2>$O/r50.err
chk $? r50; tail -1 $O/r50.log | cut -c1-200
