R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_15
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -2 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
timeout -k 10 400 python -u scripts/r2/lmdb_e2e.py > $O/lmdb_e2e.json 2> $O/lmdb_e2e.err
chk $? lmdb_e2e; cat $O/lmdb_e2e.json; tail -3 $O/lmdb_e2e.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --graph off > $O/bench_eager.json 2> $O/bench_eager.err
chk $? bench_eager; cut -c1-200 $O/bench_eager.json
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_graph.json 2> $O/bench_graph.err
chk $? bench_graph; cut -c1-200 $O/bench_graph.json; tail -3 $O/bench_graph.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --ddp --graph on > $O/bench_ddp_graph.json 2> $O/bench_ddp_graph.err
chk $? bench_ddp_graph; cut -c1-200 $O/bench_ddp_graph.json; tail -3 $O/bench_ddp_graph.err
