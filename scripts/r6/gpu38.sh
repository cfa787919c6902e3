#!/bin/bash
# (1) BN apply full grid: the norm / model GPU tests; (2) ViT-B/16: LayerNorm grid sizes A/B (alternated)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_38; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_r2_correctness.py tests/test_gpu_res_carrier.py tests/test_gpu_gxf.py tests/test_gpu_layernorm.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for cfg in 2048:512 100000:512 100000:1024 100000:2048; do
f=${cfg%:*}; b=${cfg#*:}
TBAMD_LN_FWD_WG=$f TBAMD_LN_BWD_WG=$b timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/v_${f}_${b}_$i.json 2> $O/v_${f}_${b}_$i.err || exit $?
echo "lnfwd=$f lnbwd=$b $(python3 -c "import json;d=json.load(open('$O/v_${f}_${b}_$i.json'));print(d['value'],d['ms_per_step'])")"
done
done
