#!/bin/bash
# final tree: the DDP wrapper on a 1-rank RCCL group (hooks, buckets, all-reduce, finalize all run) through
# torch.distributed.run as the driver launches N>1, then the bare N=1 step on the same box
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_82; mkdir -p $O; cd $R
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --ddp --steps 20 --warmup 5 > $O/ddp.json 2> $O/ddp.err || { tail -20 $O/ddp.err; exit 1; }
echo "ddp1 $(python3 -c "import json;d=json.load(open('$O/ddp.json'));print(d['value'],d['ms_per_step'],d['config']['ddp_wrapper'],d['final_loss'])")"
grep "ddp buckets" $O/ddp.err || true
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err || exit $?
echo "n1 $(python3 -c "import json;d=json.load(open('$O/n1.json'));print(d['value'],d['ms_per_step'],d['final_loss'])")"
