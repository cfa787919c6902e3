R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r34
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
for cfg in 64,64 16,256 32,128 8,512 64,64; do
  TBAMD_COLSUM=$cfg timeout -k 10 300 python bench.py --steps 30 --warmup 5 > $O/bench_$cfg.log 2>$O/bench_$cfg.err
  chk $? bench_$cfg; tail -1 $O/bench_$cfg.log | cut -c100-200
done
