# round-2 closing check after the LN-backward prefetch: full GPU suite, smoke, ResNet-50 / ViT / AdaIN / DCGAN benches
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_45
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
timeout -k 10 120 python __graft_entry__.py > $O/smoke.log 2>&1
chk $? smoke; tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cut -c1-200 $O/bench.json
timeout -k 10 300 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-200 $O/adain_native.json
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode native > $O/dcgan.json 2> $O/dcgan.err
chk $? dcgan; cut -c1-200 $O/dcgan.json
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 12 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cut -c1-200 $O/vit.json
kill $HB
