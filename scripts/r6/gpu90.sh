#!/bin/bash
# side stream made before the RCCL group is replaced at init (distributed.py -> streams.on_process_group_init);
# queue / stream / DDP tests, then --ddp bench through torchrun
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_90; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_ddp_queue.py tests/test_gpu_streams.py tests/test_gpu_ddp.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 1 --ddp --steps 20 --warmup 5 > $O/trun.out 2> $O/trun.err || { tail -20 $O/trun.err; exit 1; }
echo "torchrun ddp lines=$(wc -l < $O/trun.out) $(python3 -c "import json;d=json.load(open('$O/trun.out'));print(d['value'],d['ms_per_step'])")"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/plain.out 2> $O/plain.err || exit $?
echo "plain lines=$(wc -l < $O/plain.out) $(python3 -c "import json;d=json.load(open('$O/plain.out'));print(d['value'],d['ms_per_step'])")"
