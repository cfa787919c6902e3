#!/bin/bash
# closing check of the round-3 tree: full GPU suite, smoke, headline bench, ViT; then the tiny-channel
# weight-gradient re-tune of online bf16 / fp32 with an A/B against the shipped routes
set -o pipefail
O=gpurun_out/r3_40; mkdir -p $O
( while sleep 20; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1 ; chk $? pytest; tail -2 $O/pytest.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.err 2>&1; chk $? smoke; tail -1 $O/smoke.err
timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 10 > $O/r50.log 2>$O/r50.err; chk $? r50; tail -1 $O/r50.log | cut -c1-200
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-160
tune() {
TBAMD_CONV_ROUTES=none TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload $1 --batch $2 --size 256 --mode $3 --steps 20 --warmup 5 --save-routes $O/routes_$1_$3.json > $O/$1_$3_tuned.log 2>$O/$1_$3_tuned.err; chk $? $1_$3_tuned; tail -1 $O/$1_$3_tuned.log | cut -c1-140; grep "miopen (\|tinyhalo" $O/$1_$3_tuned.err | cut -c1-220
}
tune online 8 native
tune online 8 native32
timeout -k 10 300 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --mode stock --steps 30 --warmup 5 > $O/online_stock.log 2>$O/online_stock.err; chk $? online_stock; tail -1 $O/online_stock.log | cut -c1-140
