R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r26
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest; tail -2 $O/pytest_gpu.log
[ "$(grep -c failed $O/pytest_gpu.log)" = "0" ] || exit 1
for m in native; do
  timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode $m --steps 20 --warmup 4 > $O/nst_$m.log 2>$O/nst_$m.err
  chk $? nst_$m; tail -1 $O/nst_$m.log | cut -c1-200
done
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode native --graph --steps 20 --warmup 4 > $O/nst_graph.log 2>$O/nst_graph.err
chk $? nst_graph; tail -1 $O/nst_graph.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_nst -o run -- python3 $R/scripts/bench_workloads.py --workload nst --mode native --steps 10 --warmup 3 > $R/$O/prof_nst.log 2>&1
chk $? prof_nst
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err
chk $? bench; tail -1 $O/bench.log | cut -c1-200
