#!/bin/bash
# ViT-B/16 b128 GEMM epilogue knobs re-checked on the closing tree (alternated)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_70; mkdir -p $O; cd $R
run() { env "$@" timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/v.json 2> $O/v.err || exit $?; python3 -c "import json;d=json.load(open('$O/v.json'));print(d['value'],d['ms_per_step'])"; }
for i in 1 2; do
echo "default            $(run X=1)"
echo "lds_epi=0          $(run TBAMD_GEMM8_LDS_EPI=0)"
echo "gelu_bwd_nt=0      $(run TBAMD_GELU_BWD_NT=0)"
done
