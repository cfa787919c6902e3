# VIRT (reflect / upsample) addressing on the 64-channel kernels; generic conv tests; online + AdaIN benches
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_22
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
# progress marker for the long first (autotuning / MIOpen find) steps; every step keeps its own timeout
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_any.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest.log | head -80; kill $HB; exit 1; }
TBAMD_TUNE_LOG=1 timeout -k 10 400 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode native --save-routes $O/routes_online.json > $O/online_native.json 2> $O/online_native.err
chk $? online_native; cut -c1-220 $O/online_native.json; grep -c "native64" $O/online_native.err
TBAMD_TUNE_LOG=1 timeout -k 10 600 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native --save-routes $O/routes_adain.json > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-220 $O/adain_native.json
timeout -k 10 500 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode stock > $O/adain_stock.json 2> $O/adain_stock.err
chk $? adain_stock; cut -c1-220 $O/adain_stock.json
kill $HB
