R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q > gpurun_out/pytest14.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest14.log
(cd scripts && timeout -k 10 400 python conv_tune.py > ../gpurun_out/conv_tune14.log 2>&1)
echo "tune rc=$?"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench14.log 2>gpurun_out/bench14.err
echo "bench rc=$?"; tail -1 gpurun_out/bench14.log
