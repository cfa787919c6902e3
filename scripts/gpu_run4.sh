R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
set -e
timeout -k 10 600 python scripts/conv_bench.py --native > gpurun_out/conv_bench_native.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench4 -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_bench4.log 2>&1
