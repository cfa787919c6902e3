R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r25
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_nst -o run -- python3 $R/scripts/bench_workloads.py --workload nst --mode native --steps 10 --warmup 3 > $R/$O/prof_nst.log 2>&1
chk $? prof_nst
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_dcgan -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --mode native --steps 10 --warmup 3 > $R/$O/prof_dcgan.log 2>&1
chk $? prof_dcgan
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_nst_stock -o run -- python3 $R/scripts/bench_workloads.py --workload nst --mode stock --steps 10 --warmup 3 > $R/$O/prof_nst_stock.log 2>&1
chk $? prof_nst_stock
