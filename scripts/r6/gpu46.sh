#!/bin/bash
# input-gradient epilogue kernels on 64-pixel tiles (TBAMD_CONV_EPI_BN64): carrier / GXF tests, step A/B alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_46; mkdir -p $O; cd $R
TBAMD_CONV_EPI_BN64=1 timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_res_carrier.py tests/test_gpu_kernels.py > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^(FAILED|ERROR)" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
for v in 0 1; do
TBAMD_CONV_EPI_BN64=$v timeout -k 10 300 python bench.py --steps 30 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || exit $?
echo "epi_bn64=$v $(python3 -c "import json;d=json.load(open('$O/b_${v}_$i.json'));print(d['value'],d['ms_per_step'])")"
done
done
