R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q > gpurun_out/pytest15.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/pytest15.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench15.log 2>gpurun_out/bench15.err
echo "bench rc=$?"; tail -1 gpurun_out/bench15.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof15 -o run -- python $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof15.log 2>&1
echo "prof rc=$?"
