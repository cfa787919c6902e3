R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python scripts/dbg_fusion.py > gpurun_out/dbg9.log 2>&1
echo "dbg rc=$?"; grep -v amdgpu.ids gpurun_out/dbg9.log | tail -8
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q > gpurun_out/pytest9.log 2>&1
echo "pytest rc=$?"; tail -6 gpurun_out/pytest9.log
timeout -k 10 300 python scripts/bn_bench.py > gpurun_out/bn_bench9.log 2>&1
echo "bn rc=$?"; tail -1 gpurun_out/bn_bench9.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench9.log 2>gpurun_out/bench9.err
echo "bench rc=$?"; tail -1 gpurun_out/bench9.log
