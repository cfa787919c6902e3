R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest16.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/pytest16.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench16.log 2>gpurun_out/bench16.err || exit 1
echo "bench ok"; tail -1 gpurun_out/bench16.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof16 -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof16.log 2>&1
echo "prof rc=$?"
