#!/bin/bash
# rebuilt-container sanity: the driver's bench invocation x2, then multi-rank RCCL with 2 / 4 ranks sharing cuda:0
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_29; mkdir -p $O; cd $R
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
cut -c1-200 $O/bench_$i.json
done
for n in 2 4; do
timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node $n --master-addr 127.0.0.1 \
  --master-port 2951$n scripts/tools/rccl_shared_gpu_probe.py > $O/rccl_shared_$n.log 2>&1; rc=$?
grep -E "rank|Error|error" $O/rccl_shared_$n.log | head -20; echo "rccl n=$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
