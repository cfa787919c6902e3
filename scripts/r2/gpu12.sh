R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_12
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 240 python -u -m pytest tests/test_gpu_conv_any.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
timeout -k 10 300 python -u scripts/r2/conv_any_bench.py > $O/bench.jsonl 2> $O/bench.err
chk $? bench; cat $O/bench.jsonl
