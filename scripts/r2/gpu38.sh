# s_setprio 3 in every single-stage conv kernel (default now) + wgrad A/B (TBAMD_WGRAD_PRIO); conv tests
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_38
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_r2_correctness.py tests/test_gpu_conv_any.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
for p in 0 3 0 3; do
  TBAMD_WGRAD_PRIO=$p timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_w$p.json 2> $O/bench_w$p.err
  chk $? bench_w$p; cut -c1-120 $O/bench_w$p.json
done
