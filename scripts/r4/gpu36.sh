#!/bin/bash
# collect the route / tile decisions of ResNet-18/34/101/152 and ViT-S/16 (MIOpen excluded) for the shipped tables
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_36; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
export TBAMD_CONV_NO_MIOPEN=1
for m in resnet18 resnet34 resnet101 resnet152; do
TBAMD_CONV_SAVE=$O/routes_$m.json TBAMD_GEMM_SAVE=$O/tiles_$m.json timeout -k 10 400 python bench.py --model $m --steps 3 --warmup 4 > $O/$m.log 2>$O/$m.err; chk $? $m
done
TBAMD_CONV_SAVE=$O/routes_vits.json TBAMD_GEMM_SAVE=$O/tiles_vits.json timeout -k 10 400 python bench.py --model vit_s_16 --batch 128 --steps 3 --warmup 4 > $O/vits.log 2>$O/vits.err; chk $? vits
ls -la $O/*.json
echo final rc=0
