R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -k "conv" > gpurun_out/pytest13.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/pytest13.log
cd scripts && timeout -k 10 400 python conv_tune.py > ../gpurun_out/conv_tune13.log 2>&1
echo "tune rc=$?"
