# narrow-output conv (tests + AdaIN / online NST benches with routes), AdaIN + DCGAN kernel summaries
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_29
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_any.py tests/test_gpu_aux_ops.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
TBAMD_TUNE_LOG=1 timeout -k 10 400 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-200 $O/adain_native.json; grep "conv-tune.*9, 9" $O/adain_native.err
TBAMD_TUNE_LOG=1 timeout -k 10 400 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode native > $O/online_native.json 2> $O/online_native.err
chk $? online_native; cut -c1-200 $O/online_native.json; grep "conv-tune.*9, 9" $O/online_native.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/p_adain -o run -- python3 $R/scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 4 --warmup 3 --mode native > $R/$O/p_adain.json 2> $R/$O/p_adain.err
chk $? p_adain
python3 $R/scripts/dbstats.py $R/$O/p_adain/run_results.db --steps 3 --marker adamw_mt_k --top 40 --width 110 > $R/$O/adain_kernels.txt 2>&1; rm -f $R/$O/p_adain/run_results.db
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/p_dcgan -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --steps 4 --warmup 3 --mode native > $R/$O/p_dcgan.json 2> $R/$O/p_dcgan.err
chk $? p_dcgan
python3 $R/scripts/dbstats.py $R/$O/p_dcgan/run_results.db --steps 3 --markers-per-step 2 --marker adamw_mt_k --top 40 --width 110 > $R/$O/dcgan_kernels.txt 2>&1; rm -f $R/$O/p_dcgan/run_results.db
du -sh $R/$O
kill $HB
