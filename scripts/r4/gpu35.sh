#!/bin/bash
# the ResNet family beyond the headline (BasicBlock 18/34, Bottleneck 101/152) and ViT-S/16, native vs
# the stock PyTorch-ROCm stack, b256 bf16 (ViT-S b128)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_35; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for m in resnet18 resnet34 resnet101 resnet152; do
timeout -k 10 400 python bench.py --model $m --steps 15 --warmup 6 > $O/${m}_nat.log 2>$O/${m}_nat.err; chk $? ${m}_nat; echo "${m}_nat $(v ${m}_nat)"
timeout -k 10 400 python bench.py --model $m --mode stock --steps 10 --warmup 4 > $O/${m}_stock.log 2>$O/${m}_stock.err; chk $? ${m}_stock; echo "${m}_stock $(v ${m}_stock)"
done
timeout -k 10 400 python bench.py --model vit_s_16 --batch 128 --steps 15 --warmup 6 > $O/vits_nat.log 2>$O/vits_nat.err; chk $? vits_nat; echo "vits_nat $(v vits_nat)"
timeout -k 10 400 python bench.py --model vit_s_16 --batch 128 --mode stock --steps 10 --warmup 4 > $O/vits_stock.log 2>$O/vits_stock.err; chk $? vits_stock; echo "vits_stock $(v vits_stock)"
echo final rc=0
