R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=gpurun_out/r29
mkdir -p $R/$O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_rn50 -o run -- python3 $R/bench.py --steps 6 --warmup 4 > $R/$O/prof_rn50.log 2>&1
echo "prof rc=$?"
