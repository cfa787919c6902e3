set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python scripts/probe_gpu.py --steps 10 > gpurun_out/probe.log 2>&1
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ours -o run --output-format csv -- python3 $R/scripts/probe_gpu.py --no-check --only ours --steps 5 --warmup 2 > $R/gpurun_out/prof_ours.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stock -o run --output-format csv -- python3 $R/scripts/probe_gpu.py --no-check --only stock --steps 5 --warmup 2 > $R/gpurun_out/prof_stock.log 2>&1
