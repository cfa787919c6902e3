#!/bin/bash
# why does the 1-rank RCCL DDP wrapper cost 12 % on the final tree (r6_82)?  host submission vs wall, plain vs --ddp,
# alternated; then a kernel trace of the --ddp step (main-stream gaps, RCCL kernels)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_83; mkdir -p $O; cd $R
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err || exit $?
echo "plain $(python3 -c "import json;d=json.load(open('$O/n1.json'));print(d['value'],d['ms_per_step'])") $(grep 'host submit' $O/n1.err)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2953$i bench.py --gpus 1 --ddp --steps 20 --warmup 5 > $O/ddp.out 2> $O/ddp.err || { tail -20 $O/ddp.err; exit 1; }
echo "ddp $(grep '^{' $O/ddp.out | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])") $(grep 'host submit' $O/ddp.err)"
done
grep -v '^{' $O/ddp.out | head -5 > $O/ddp_stdout_nonjson.txt || true
