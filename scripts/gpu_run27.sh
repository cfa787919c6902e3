R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r27
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_examples.py -v --timeout 150 --timeout-method thread > $O/pytest_ex.log 2>&1
chk $? pytest_ex; grep -E "PASSED|FAILED|ERROR" $O/pytest_ex.log | cut -c1-150
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 20 --warmup 4 > $O/dcgan_native.log 2>$O/dcgan_native.err
chk $? dcgan; tail -1 $O/dcgan_native.log | cut -c1-200
