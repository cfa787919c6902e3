#!/bin/bash
# GXF: fp32-referenced bottleneck test after the materialize fix; kernel traces GXF off / on
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_31; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_gxf.py -k "pair or deferred" > $O/test_gxf.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert" $O/test_gxf.log | tail -30
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
TBAMD_BN_GXF=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$v -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr$v.err 2>&1 || exit $?
python3 $R/scripts/steady.py $(find $O/tr$v -name '*kernel_trace.csv' | head -1) 3 1 60 > $O/steady$v.txt
head -3 $O/steady$v.txt
done
