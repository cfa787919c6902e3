# s_setprio on the single-stage conv MFMA phase: per-shape sweep + whole-step A/B
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_37
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
WGRAD=0 timeout -k 10 300 python -u scripts/r2/conv_bk_tune.py > $O/tune.jsonl 2> $O/tune.err
chk $? tune; tail -1 $O/tune.jsonl | cut -c1-300
for p in 0 1 0 1 3; do
  TBAMD_CONV_PRIO=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_p$p.json 2> $O/bench_p$p.err
  chk $? bench_p$p; cut -c1-120 $O/bench_p$p.json
done
