# flip cache: test + ResNet bench + kernel trace
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_10
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 240 python -u -m pytest tests/test_gpu_r2_correctness.py tests/test_gpu_kernels.py tests/test_gpu_examples.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest.log | head -80; exit 1; }
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cut -c1-200 $O/bench.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r50 -- python bench.py --steps 4 --warmup 3 > $O/prof.log 2>&1
chk $? prof
python scripts/steady.py $O/prof/r50_kernel_trace.csv 3 > $O/r50_steady.txt; head -45 $O/r50_steady.txt
