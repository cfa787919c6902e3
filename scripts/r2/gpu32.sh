# tiny-input-channel conv: tests; AdaIN / online / DCGAN benches with the new routes; AdaIN kernel summary
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_32
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_any.py tests/test_gpu_nativize.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-200 $O/adain_native.json; grep "conv-tune.*fwd.*any" $O/adain_native.err
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode native > $O/online_native.json 2> $O/online_native.err
chk $? online_native; cut -c1-200 $O/online_native.json; grep "conv-tune.*fwd.*any" $O/online_native.err
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode native > $O/dcgan.json 2> $O/dcgan.err
chk $? dcgan; cut -c1-200 $O/dcgan.json; grep "conv-tune" $O/dcgan.err | grep -v "> native" | cut -c1-250
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/p_adain -o run -- python3 $R/scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 4 --warmup 3 --mode native > $R/$O/p_adain.json 2> $R/$O/p_adain.err
chk $? p_adain
python3 $R/scripts/dbstats.py $R/$O/p_adain/run_results.db --steps 3 --marker adamw_mt_k --top 40 --width 110 > $R/$O/adain_kernels.txt 2>&1; rm -f $R/$O/p_adain/run_results.db
kill $HB
