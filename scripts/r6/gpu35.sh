#!/bin/bash
# ViT-B/16 b128: host-bound? per-step spread + host submit, eager vs hipGraph replay (alternated)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_35; mkdir -p $O; cd $R
for i in 1 2; do
for gr in off on; do
TBAMD_BENCH_STEPTIMES=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 30 --warmup 8 --graph $gr > $O/vit_$gr$i.json 2> $O/vit_$gr$i.err || exit $?
echo "graph=$gr $(python3 -c "import json;d=json.load(open('$O/vit_$gr$i.json'));print(d['value'],d['ms_per_step'])") $(grep -E 'host submit' $O/vit_$gr$i.err) $(grep per-step $O/vit_$gr$i.err | cut -c1-80)"
done
done
