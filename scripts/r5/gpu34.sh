#!/bin/bash
# ViT-B/16 at batch 128 (the verdict's config): step x2, then the whole-step PMC profile
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_34; mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/b128_$i.log 2>$O/b128_$i.err || { echo "bench failed"; tail -5 $O/b128_$i.err; exit 1; }
tail -1 $O/b128_$i.log | cut -c1-200
done
PROF_OUT=r5_34/prof BENCH_ARGS="--model vit_b_16 --batch 128" bash $R/scripts/repro/profile_step.sh || exit 1
echo final rc=0
