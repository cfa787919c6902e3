R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_14
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 240 python -u -m pytest tests/test_gpu_conv_any.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -2 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
for M in native32 native; do
timeout -k 10 240 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode $M > $O/online_$M.json 2> $O/online_$M.err
chk $? online_$M; cut -c1-160 $O/online_$M.json
done
timeout -k 10 240 python scripts/bench_workloads.py --workload nst --size 512 --steps 10 --warmup 3 --mode native32 > $O/nst_native32.json 2> $O/nst_native32.err
chk $? nst_native32; cut -c1-160 $O/nst_native32.json
timeout -k 10 300 python -u scripts/r2/conv_any_bench.py > $O/bench.jsonl 2> $O/bench.err
chk $? bench; cat $O/bench.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_debug.py -x -q --timeout 300 --timeout-method thread > $O/pytest_debug.log 2>&1
chk $? pytest_debug; tail -3 $O/pytest_debug.log
[ "$(grep -c FAILED $O/pytest_debug.log)" = "0" ] || { grep -m3 -B5 -A30 "Error\|assert" $O/pytest_debug.log | head -60; exit 1; }
