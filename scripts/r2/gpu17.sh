# DCGAN native steady-state kernel table (why 9.07 ms vs round-1 7.6 ms)
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_17
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o dc -- python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 5 --warmup 3 --mode native > $O/prof.log 2>&1
chk $? prof
python scripts/steady.py $O/prof/dc_kernel_trace.csv 3 2 > $O/dc_steady.txt; head -60 $O/dc_steady.txt
