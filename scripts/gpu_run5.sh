R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -k "conv" > gpurun_out/pytest_conv.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python scripts/conv_bench.py --native-only --dgrad > gpurun_out/conv_bench_v2.log 2>&1
