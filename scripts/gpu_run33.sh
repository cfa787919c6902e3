R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r33
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_aux_ops.py -x -q --timeout 120 --timeout-method thread > $O/pytest_aux.log 2>&1
chk $? pytest_aux; tail -3 $O/pytest_aux.log
[ "$(grep -c failed $O/pytest_aux.log)" = "0" ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
chk $? smoke; tail -1 $O/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest; tail -2 $O/pytest_gpu.log
for w in vae; do
  timeout -k 10 200 python scripts/bench_workloads.py --workload $w --mode native --graph --batch 256 --steps 50 --warmup 5 > $O/${w}_graph.log 2>$O/${w}_graph.err
  chk $? ${w}_graph; tail -1 $O/${w}_graph.log | cut -c1-150
done
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode native --graph --steps 20 --warmup 4 > $O/nst_graph.log 2>$O/nst_graph.err
chk $? nst_graph; tail -1 $O/nst_graph.log | cut -c1-150
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err
chk $? bench; tail -1 $O/bench.log | cut -c1-220
