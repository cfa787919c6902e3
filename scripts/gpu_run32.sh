R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r32
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
chk $? smoke; tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest; tail -2 $O/pytest_gpu.log
for w in lenet vae; do
  timeout -k 10 200 python scripts/bench_workloads.py --workload $w --mode native --graph --batch 256 --steps 50 --warmup 5 > $O/${w}_graph.log 2>$O/${w}_graph.err
  chk $? ${w}_graph; tail -1 $O/${w}_graph.log | cut -c1-150
done
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode native --graph --steps 20 --warmup 4 > $O/nst_graph.log 2>$O/nst_graph.err
chk $? nst_graph; tail -1 $O/nst_graph.log | cut -c1-150
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 20 --warmup 4 > $O/dcgan.log 2>$O/dcgan.err
chk $? dcgan; tail -1 $O/dcgan.log | cut -c1-150
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 3 > $O/vit.log 2>$O/vit.err
chk $? vit; tail -1 $O/vit.log | cut -c1-150
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err
chk $? bench; tail -1 $O/bench.log | cut -c1-150
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --batch 32 --steps 3 --warmup 2 > $O/ddp2.log 2>$O/ddp2.err
chk $? ddp2; tail -1 $O/ddp2.log | cut -c1-150
