#!/bin/bash
# re-tune the ViT-B/16 b128 GEMM rows with hipBLASLt a candidate (the shipped rows predate it), A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_17; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
python scripts/r5/tiles_drop.py $O/tiles_in.json tn
TBAMD_GEMM_TILES=$O/tiles_in.json TBAMD_GEMM_SAVE=$O/tiles_tuned.json TBAMD_TUNE_LOG=1 timeout -k 10 400 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 3 > $O/tune.log 2>$O/tune.err; chk $? tune; echo "tune $(v tune)"
grep "gemm-tune" $O/tune.err | head -40
cp torchbooster_amd/ops/gemm_tiles_gfx950.json $O/tiles_old.json
python scripts/merge_tiles.py $O/tiles_tuned.json && cp torchbooster_amd/ops/gemm_tiles_gfx950.json $O/merged_tiles.json
for i in 1 2; do
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/new_$i.log 2>$O/new_$i.err; chk $? new_$i; echo "new_$i $(v new_$i)"
TBAMD_GEMM_TILES=$O/tiles_old.json timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/old_$i.log 2>$O/old_$i.err; chk $? old_$i; echo "old_$i $(v old_$i)"
done
echo final rc=0
