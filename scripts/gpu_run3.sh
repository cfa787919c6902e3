set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python scripts/conv_bench.py > gpurun_out/conv_bench.log 2>&1
