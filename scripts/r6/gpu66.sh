#!/bin/bash
# conv backward launch order: input gradient queued before the side-stream weight gradient (TBAMD_DGRAD_FIRST)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_66; mkdir -p $O; cd $R
TBAMD_DGRAD_FIRST=1 timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_res_carrier.py tests/test_gpu_streams.py > $O/tests.log 2>&1; rc=$?
tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
for v in 0 1; do
TBAMD_DGRAD_FIRST=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "dgrad_first=$v $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
