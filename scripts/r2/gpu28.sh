# vectorised BN column-sum finalize (tests + A/B on the bench); AdaIN native/stock and DCGAN kernel profiles
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_28
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 400 python -u -m pytest tests/test_gpu_aux_ops.py tests/test_gpu_kernels.py tests/test_gpu_r2_correctness.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
for v in 0 1 0 1; do
  TBAMD_COLSUM_SCALAR=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench_scalar$v.json 2> $O/bench_scalar$v.err
  chk $? bench_scalar$v; cut -c1-150 $O/bench_scalar$v.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $R/$O/r50prof -o run -- python3 $R/bench.py --steps 5 --warmup 5 > $R/$O/r50prof.log 2>&1
chk $? r50prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/adain_native -o run -- python3 $R/scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 4 --warmup 3 --mode native > $R/$O/adain_native.json 2> $R/$O/adain_native.err
chk $? adain_native; cut -c1-200 $R/$O/adain_native.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/adain_stock -o run -- python3 $R/scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 4 --warmup 3 --mode stock > $R/$O/adain_stock.json 2> $R/$O/adain_stock.err
chk $? adain_stock; cut -c1-200 $R/$O/adain_stock.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/dcgan -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --steps 4 --warmup 3 --mode native > $R/$O/dcgan.json 2> $R/$O/dcgan.err
chk $? dcgan; cut -c1-200 $R/$O/dcgan.json
kill $HB
