#!/bin/bash
# native vs stock PyTorch-ROCm on ONE box for the family (refreshes the round-4 stock column);
# MIOpen compiles on first use on a fresh box: heartbeat every 30 s
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_64; mkdir -p $O; cd $R
( while sleep 30; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
v() { python3 -c "import json;d=json.load(open('$1'));print(d['value'])"; }
for m in resnet18 resnet34 resnet101 resnet152; do
for mode in native stock; do
timeout -k 10 900 python bench.py --model $m --mode $mode --steps 10 --warmup 3 > $O/${m}_$mode.json 2> $O/${m}_$mode.err || exit $?
done
echo "$m native $(v $O/${m}_native.json) stock $(v $O/${m}_stock.json)"
done
for m in vit_s_16 vit_b_16; do
for mode in native stock; do
timeout -k 10 900 python bench.py --model $m --batch 128 --mode $mode --steps 10 --warmup 5 > $O/${m}_$mode.json 2> $O/${m}_$mode.err || exit $?
done
echo "$m native $(v $O/${m}_native.json) stock $(v $O/${m}_stock.json)"
done
for mode in native stock; do
timeout -k 10 900 python scripts/bench_workloads.py --workload dcgan --mode $mode --steps 40 --warmup 8 > $O/dcgan_$mode.json 2> $O/dcgan_$mode.err || exit $?
done
echo "dcgan native $(tail -1 $O/dcgan_native.json | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])') stock $(tail -1 $O/dcgan_stock.json | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["value"])')"
