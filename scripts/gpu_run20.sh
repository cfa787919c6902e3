R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r20
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $O/pytest.log
timeout -k 10 300 python scripts/bench_workloads.py --workload vit --mode native --batch 128 --steps 10 --warmup 3 > $O/vit_native.log 2>$O/vit_native.err || exit 1
tail -1 $O/vit_native.log
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop.csv timeout -k 10 500 python scripts/bench_workloads.py --workload vit --mode native --batch 128 --steps 10 --warmup 3 > $O/vit_tuned.log 2>$O/vit_tuned.err || exit 1
tail -1 $O/vit_tuned.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 6 --warmup 3 > $R/$O/prof_vit.log 2>&1
echo "prof rc=$?"
