# generic conv: stride-phase dgrad, 4-step wgrad, window GEMM, colsum bias grads; DCGAN
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_18
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_any.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest.log | head -80; exit 1; }
TBAMD_TUNE_LOG=1 timeout -k 10 240 python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 20 --warmup 3 --mode native > $O/dcgan_native.json 2> $O/dcgan_native.err
chk $? dcgan; cut -c1-200 $O/dcgan_native.json; grep conv-tune $O/dcgan_native.err | grep "any"
timeout -k 10 240 python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 20 --warmup 3 --graph > $O/dcgan_graph.json 2> $O/dcgan_graph.err
chk $? dcgan_graph; cut -c1-200 $O/dcgan_graph.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o dc -- python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 5 --warmup 3 --mode native > $O/prof.log 2>&1
chk $? prof
python scripts/steady.py $O/prof/dc_kernel_trace.csv 3 2 > $O/dc_steady.txt; head -40 $O/dc_steady.txt
