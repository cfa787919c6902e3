#!/bin/bash
# ViT-S/16: the merged family tiles vs the table before the merge (first-use tuning), alternated
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_38; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2; do
timeout -k 10 300 python bench.py --model vit_s_16 --batch 128 --steps 15 --warmup 6 > $O/new$i.log 2>$O/new$i.err; chk $? new$i; echo "new$i $(v new$i)"
TBAMD_GEMM_TILES=$R/scripts/r4/tiles_before_family.json timeout -k 10 300 python bench.py --model vit_s_16 --batch 128 --steps 15 --warmup 6 > $O/old$i.log 2>$O/old$i.err; chk $? old$i; echo "old$i $(v old$i)"
done
echo final rc=0
