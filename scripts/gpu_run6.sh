# wgrad kernel numerics + per-shape timing, then the end-to-end bench
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -k "conv" > gpurun_out/pytest_conv6.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/pytest_conv6.log
timeout -k 10 300 python scripts/conv_bench.py --native-only --dgrad > gpurun_out/conv_bench_v6.log 2>&1
echo "conv_bench rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench6.log 2>&1
echo "bench rc=$?"
tail -2 gpurun_out/bench6.log
