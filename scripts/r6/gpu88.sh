#!/bin/bash
# the DDP side-stream queue fix on the other DDP configs: ViT-B/16 b128 and ResNet-101, plain vs --ddp (auto) vs
# --ddp with the old normal-priority side stream, alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_88; mkdir -p $O; cd $R
run() { n=$1; shift; env $E timeout -k 10 300 python bench.py --warmup 6 "$@" > $O/$n.out 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
echo "$n $(python3 -c "import json;d=json.load(open('$O/$n.out'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2; do
E=A=1 run vit_plain --model vit_b_16 --batch 128 --steps 20
E=A=1 run vit_ddp --model vit_b_16 --batch 128 --steps 20 --ddp
E=TBAMD_SIDE_PRIORITY=normal run vit_ddp_old --model vit_b_16 --batch 128 --steps 20 --ddp
done
E=A=1 run r101_plain --model resnet101 --steps 15
E=A=1 run r101_ddp --model resnet101 --steps 15 --ddp
E=TBAMD_SIDE_PRIORITY=normal run r101_ddp_old --model resnet101 --steps 15 --ddp
