R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r24
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_graph_step.py tests/test_gpu_layernorm.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -2 $O/pytest.log
[ "$(grep -c failed $O/pytest.log)" = "0" ] || exit 1
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode native --graph --steps 20 --warmup 4 > $O/nst_graph.log 2>$O/nst_graph.err
chk $? nst_graph; tail -1 $O/nst_graph.log | cut -c1-200
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 3 > $O/vit.log 2>$O/vit.err
chk $? vit; tail -1 $O/vit.log | cut -c1-200
