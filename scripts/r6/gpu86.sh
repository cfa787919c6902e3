#!/bin/bash
# side stream low priority under RCCL (auto): queue test, DDP / stream tests, then plain vs --ddp (1-rank RCCL) alternated,
# torchrun --ddp with stdout checked to be exactly one JSON line, and a 2-rank gloo torchrun rehearsal
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_86; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_ddp_queue.py tests/test_gpu_streams.py tests/test_gpu_ddp.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
run() { n=$1; shift; timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > $O/$n.out 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
echo "$n lines=$(wc -l < $O/$n.out) $(python3 -c "import json;d=json.load(open('$O/$n.out'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2; do
run plain
run ddp --ddp
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --ddp --steps 20 --warmup 5 > $O/trun.out 2> $O/trun.err || { tail -20 $O/trun.err; exit 1; }
echo "torchrun ddp lines=$(wc -l < $O/trun.out) $(python3 -c "import json;d=json.load(open('$O/trun.out'));print(d['value'],d['ms_per_step'],d['config']['ddp_wrapper'])")"
TBAMD_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --steps 3 --warmup 2 --batch 32 > $O/gloo2.out 2> $O/gloo2.err || { tail -20 $O/gloo2.err; exit 1; }
echo "gloo2 lines=$(wc -l < $O/gloo2.out) $(python3 -c "import json;d=json.load(open('$O/gloo2.out'));print(d['n_gpus'],d['config']['parallelism'],d['config']['backend'])")"
