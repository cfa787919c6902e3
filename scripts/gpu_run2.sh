set -e
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.log 2>&1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --mode stock > gpurun_out/bench_stock.log 2>&1
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/prof_bench.log 2>&1
