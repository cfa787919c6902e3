R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r21
mkdir -p $O
# stop on faults / aborts / timeouts (124 timeout, 134 abort, 137 kill, 139 segv); tolerate plain errors (1)
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest; tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err
chk $? bench; tail -1 $O/bench.log
# 2-rank DDP rehearsal on one GPU (gloo collectives, both ranks on cuda:0)
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --batch 32 --steps 3 --warmup 2 > $O/ddp2.log 2>$O/ddp2.err
chk $? ddp2; tail -1 $O/ddp2.log
for w in lenet vae; do
  for m in native stock; do
    timeout -k 10 200 python scripts/bench_workloads.py --workload $w --mode $m --batch 256 --steps 50 --warmup 5 > $O/${w}_$m.log 2>$O/${w}_$m.err
    chk $? ${w}_$m; tail -1 $O/${w}_$m.log | cut -c1-200
  done
  timeout -k 10 200 python scripts/bench_workloads.py --workload $w --mode native --graph --batch 256 --steps 50 --warmup 5 > $O/${w}_graph.log 2>$O/${w}_graph.err
  chk $? ${w}_graph; tail -1 $O/${w}_graph.log | cut -c1-200
done
