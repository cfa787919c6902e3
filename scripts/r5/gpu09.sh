#!/bin/bash
# big-tile conv route candidates: kernel tests, re-tune the ResNet-50 b256 rows, A/B with and without
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_09; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_big.py > $O/t.log 2>$O/t.err; rc=$?; tail -3 $O/t.log; chk $rc t
python scripts/r5/routes_drop.py $O/routes_in.json
TBAMD_CONV_ROUTES=$O/routes_in.json TBAMD_CONV_SAVE=$O/routes_tuned.json TBAMD_TUNE_LOG=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/tune.log 2>$O/tune.err; chk $? tune; echo "tune $(v tune)"
python scripts/merge_routes.py $O/routes_tuned.json && cp torchbooster_amd/ops/conv_routes_gfx950.json $O/merged_routes.json
grep -c "big" $O/merged_routes.json
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/new_$i.log 2>$O/new_$i.err; chk $? new_$i; echo "new_$i $(v new_$i)"
TBAMD_CONV_BIG_ROUTES=0 timeout -k 10 300 python bench.py > $O/off_$i.log 2>$O/off_$i.err; chk $? off_$i; echo "off_$i $(v off_$i)"
done
echo final rc=0
