#!/bin/bash
# ResNet-50 conv routes re-tuned on the round-4 kernels (no shipped table, MIOpen excluded) vs the
# shipped table, alternated; the fresh decisions are saved for scripts/merge_routes.py
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_18; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
TBAMD_CONV_ROUTES=none TBAMD_CONV_NO_MIOPEN=1 TBAMD_CONV_SAVE=$O/r50_routes.json TBAMD_TUNE_LOG=1 timeout -k 10 600 python -u bench.py --steps 30 --warmup 10 > $O/tune.log 2>$O/tune.err; chk $? tune; echo "tune $(v tune)"
grep -c "" $O/r50_routes.json
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/ship$i.log 2>$O/ship$i.err; chk $? ship$i; echo "ship$i $(v ship$i)"
TBAMD_CONV_ROUTES=$O/r50_routes.json timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/fresh$i.log 2>$O/fresh$i.err; chk $? fresh$i; echo "fresh$i $(v fresh$i)"
done
echo final rc=0
