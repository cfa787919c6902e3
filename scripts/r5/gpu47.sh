#!/bin/bash
# single-stage big-tile conv (2 workgroups/CU, epilogue overlapped) as route candidates: kernel tests,
# re-tune the stage-2..4 1x1 rows in context, A/B the merged table against the shipped one
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_47; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv_big.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; chk $rc t
cp torchbooster_amd/ops/conv_routes_gfx950.json $O/routes_shipped.json
python scripts/r5/routes_drop2.py $O/routes_in.json
TBAMD_CONV_ROUTES=$O/routes_in.json TBAMD_CONV_SAVE=$O/routes_tuned.json TBAMD_TUNE_LOG=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/tune.log 2>$O/tune.err; chk $? tune; echo "tune $(v tune)"
grep -h "s1\|big" $O/tune.err | head -40 > $O/tune_big.txt || true
python scripts/merge_routes.py $O/routes_tuned.json && cp torchbooster_amd/ops/conv_routes_gfx950.json $O/merged_routes.json
grep -o 'big[0-9x]*s1' $O/merged_routes.json | sort | uniq -c
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/new_$i.log 2>$O/new_$i.err; chk $? new_$i; echo "new_$i $(v new_$i)"
TBAMD_CONV_ROUTES=$O/routes_shipped.json timeout -k 10 300 python bench.py > $O/old_$i.log 2>$O/old_$i.err; chk $? old_$i; echo "old_$i $(v old_$i)"
done
echo final rc=0
