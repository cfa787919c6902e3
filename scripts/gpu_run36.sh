R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r36
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
for t in 1 0 1 0; do
  TBAMD_NATIVE_CONVT=$t timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 40 --warmup 6 > $O/dcgan_$t.log 2>$O/dcgan_$t.err
  chk $? dcgan_convt$t; tail -1 $O/dcgan_$t.log | cut -c1-120
done
