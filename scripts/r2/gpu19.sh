# generic conv forward: NB pixel blocks for narrow outputs, LDS-staged 16-B output stores
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_19
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_any.py tests/test_gpu_nativize.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest.log | head -80; exit 1; }
TBAMD_TUNE_LOG=1 timeout -k 10 240 python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 20 --warmup 3 --mode native > $O/dcgan_native.json 2> $O/dcgan_native.err
chk $? dcgan; cut -c1-200 $O/dcgan_native.json; grep conv-tune $O/dcgan_native.err | grep "any"
for P in native32 native; do
TBAMD_TUNE_LOG=1 timeout -k 10 240 python scripts/bench_workloads.py --workload online --steps 10 --warmup 3 --mode $P > $O/online_$P.json 2> $O/online_$P.err
chk $? online_$P; cut -c1-200 $O/online_$P.json; grep conv-tune $O/online_$P.err | grep -c miopen
done
