#!/bin/bash
# ResNet stem conv with its 4 k-tiles pipelined (TBAMD_STEM_STAGES=2|4): stem tests per variant, then step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_69; mkdir -p $O; cd $R
for v in 2 4; do
TBAMD_STEM_STAGES=$v timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu -k "stem" tests/test_gpu_kernels.py tests/test_gpu_r2_correctness.py > $O/t$v.log 2>&1; rc=$?
echo "stages=$v tests: $(tail -1 $O/t$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3; do
for v in 1 2 4; do
TBAMD_STEM_STAGES=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "stem_stages=$v $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
