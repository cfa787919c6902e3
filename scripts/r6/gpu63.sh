#!/bin/bash
# fused AdamW chunking: ~1024 workgroups (default) vs 8192 shorter ones, ResNet-50 and ViT-B/16, alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_63; mkdir -p $O; cd $R
for i in 1 2; do
for t in 1024 8192; do
TBAMD_OPT_TARGET_CHUNKS=$t timeout -k 10 300 python bench.py --steps 30 > $O/r.json 2> $O/r.err || exit $?
TBAMD_OPT_TARGET_CHUNKS=$t timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/v.json 2> $O/v.err || exit $?
echo "chunks=$t r50 $(python3 -c "import json;d=json.load(open('$O/r.json'));print(d['value'])") vit $(python3 -c "import json;d=json.load(open('$O/v.json'));print(d['value'])")"
done
done
