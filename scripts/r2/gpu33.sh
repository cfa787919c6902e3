# round-2 closing check: full GPU suite, smoke, 1-GPU bench x2, ResNet-50 kernel summary, ViT bench
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_33
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
timeout -k 10 120 python __graft_entry__.py > $O/smoke.log 2>&1
chk $? smoke; tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err
  chk $? bench$i; cut -c1-200 $O/bench$i.json
done
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cut -c1-200 $O/vit.json
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-200 $O/adain_native.json; grep "conv-tune" $O/adain_native.err | cut -c1-220
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode native > $O/online_native.json 2> $O/online_native.err
chk $? online_native; cut -c1-200 $O/online_native.json; grep "conv-tune" $O/online_native.err | cut -c1-220
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode native > $O/dcgan.json 2> $O/dcgan.err
chk $? dcgan; cut -c1-200 $O/dcgan.json; grep "conv-tune" $O/dcgan.err | grep -v "> native" | cut -c1-220
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p_r50 -o run -- python3 $R/bench.py --steps 5 --warmup 5 > $R/$O/p_r50.log 2>&1
chk $? p_r50
python3 $R/scripts/dbstats.py $R/$O/p_r50/run_results.db --steps 4 --top 50 --width 110 > $R/$O/r50_kernels.txt 2>&1; rm -f $R/$O/p_r50/run_results.db
kill $HB
