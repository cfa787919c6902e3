R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r35
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 240 python -u -m pytest tests/test_gpu_conv_transpose.py -x -v --timeout 120 --timeout-method thread > $O/pytest_convT.log 2>&1
chk $? pytest_convT; tail -3 $O/pytest_convT.log
[ "$(grep -c FAILED $O/pytest_convT.log)" = "0" ] || exit 1
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 20 --warmup 4 > $O/dcgan.log 2>$O/dcgan.err
chk $? dcgan; tail -1 $O/dcgan.log | cut -c1-200; grep "conv-tune" $O/dcgan.err | cut -c1-160 | head -40
timeout -k 10 300 python -u -m pytest tests/test_gpu_examples.py -x -q --timeout 150 --timeout-method thread > $O/pytest_examples.log 2>&1
chk $? pytest_examples; tail -2 $O/pytest_examples.log
