R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python scripts/dbg_fusion.py > gpurun_out/dbg8.log 2>&1
echo "dbg rc=$?"; cat gpurun_out/dbg8.log | grep -v amdgpu.ids
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -k "bottleneck" > gpurun_out/pytest8.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/pytest8.log
timeout -k 10 300 python scripts/bn_bench.py > gpurun_out/bn_bench8.log 2>&1
echo "bn rc=$?"
