R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q > gpurun_out/pytest12.log 2>&1
echo "pytest rc=$?"; tail -6 gpurun_out/pytest12.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench12.log 2>gpurun_out/bench12.err
echo "bench rc=$?"; tail -1 gpurun_out/bench12.log
timeout -k 10 300 python scripts/bn_bench.py > gpurun_out/bn_bench12.log 2>&1
echo "bn rc=$?"; tail -1 gpurun_out/bn_bench12.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof12 -o run -- python $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof12.log 2>&1
echo "prof rc=$?"
