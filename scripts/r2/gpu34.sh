# merged stride-2 classes spread over XCDs + narrow transposed conv: tests, ResNet-50 / DCGAN benches, R50 kernel summary
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_34
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_any.py tests/test_gpu_kernels.py tests/test_gpu_r2_correctness.py tests/test_gpu_examples.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err
  chk $? bench$i; cut -c1-200 $O/bench$i.json
done
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode native > $O/dcgan.json 2> $O/dcgan.err
chk $? dcgan; cut -c1-200 $O/dcgan.json; grep "conv-tune" $O/dcgan.err | grep -v "> native" | cut -c1-220
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode stock > $O/dcgan_stock.json 2> $O/dcgan_stock.err
chk $? dcgan_stock; cut -c1-200 $O/dcgan_stock.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p_r50 -o run -- python3 $R/bench.py --steps 5 --warmup 5 > $R/$O/p_r50.log 2>&1
chk $? p_r50
python3 $R/scripts/dbstats.py $R/$O/p_r50/run_results.db --steps 4 --top 50 --width 110 > $R/$O/r50_kernels.txt 2>&1; rm -f $R/$O/p_r50/run_results.db
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/p_dcgan -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --steps 4 --warmup 3 --mode native > $R/$O/p_dcgan.json 2> $R/$O/p_dcgan.err
chk $? p_dcgan
python3 $R/scripts/dbstats.py $R/$O/p_dcgan/run_results.db --steps 3 --markers-per-step 2 --marker adamw_mt_k --top 40 --width 110 > $R/$O/dcgan_kernels.txt 2>&1; rm -f $R/$O/p_dcgan/run_results.db
kill $HB
