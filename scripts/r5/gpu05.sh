#!/bin/bash
# (1) where the big-tile path diverges (first BN whose running mean differs); (2) ViT-B/16 on the
# round-2 tree (.bisect/r2, built in place) vs HEAD, alternated on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_05; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
TBAMD_CONV_NO_MIOPEN=1 timeout -k 10 300 python -u scripts/r5/diag_big.py 64 > $O/diag_nomio.txt 2>&1; echo "diag rc=$?"; grep -A60 "model order" $O/diag_nomio.txt | head -60
for i in 1 2; do
(cd .bisect/r2 && timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8) > $O/vit_r2_$i.log 2>$O/vit_r2_$i.err; chk $? vit_r2_$i; echo "vit_r2_$i $(v vit_r2_$i)"
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/vit_head_$i.log 2>$O/vit_head_$i.err; chk $? vit_head_$i; echo "vit_head_$i $(v vit_head_$i)"
done
echo final rc=0
