#!/bin/bash
# closing tree: stock comparator re-measured next to the native step on one box (MIOpen compiles its
# kernels on first use on a fresh box: a heartbeat line every 30 s), then the 8-rank gloo rehearsal of
# the bench.py DDP path (desync check + bf16/f32 precision probe)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_56; mkdir -p $O; cd $R
( while sleep 30; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for m in native stock native; do
timeout -k 10 900 python bench.py --mode $m --steps 20 > $O/b_$m.json 2> $O/b_$m.err || exit $?
echo "$m $(python3 -c "import json;d=json.load(open('$O/b_$m.json'));print(d['value'],d['ms_per_step'])")"
done
DDP_OUT=r6_56/ddp timeout -k 10 1200 bash scripts/repro/ddp_rehearsal.sh || exit $?
