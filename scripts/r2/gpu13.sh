# generic conv integration: tests, online/offline NST at reference fp32 and bf16 vs stock, kernel names
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_13
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv_any.py tests/test_gpu_nativize.py tests/test_gpu_examples.py tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
for M in native32 stock32 native stock; do
TBAMD_TUNE_LOG=1 timeout -k 10 240 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode $M > $O/online_$M.json 2> $O/online_$M.err
chk $? online_$M; cut -c1-200 $O/online_$M.json
done
for M in native32 stock32; do
timeout -k 10 240 python scripts/bench_workloads.py --workload nst --size 512 --steps 10 --warmup 3 --mode $M > $O/nst_$M.json 2> $O/nst_$M.err
chk $? nst_$M; cut -c1-200 $O/nst_$M.json
done
grep "conv-tune" $O/online_native32.err | head -40
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o online -- python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 3 --warmup 2 --mode native32 > $O/prof.log 2>&1
chk $? prof
python scripts/steady.py $O/prof/online_kernel_trace.csv 3 > $O/online_steady.txt; head -30 $O/online_steady.txt
