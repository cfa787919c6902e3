#!/bin/bash
# deferred BN backward apply (GXF): model tests (diagnostic print), then the step A/B (alternated)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_30; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_gxf.py -k "not kernel" > $O/test_gxf.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|assert|  [a-z0-9_.]+ +[0-9.e+-]+$" $O/test_gxf.log | tail -80
for i in 1 2; do
for v in 0 1; do
TBAMD_BN_GXF=$v timeout -k 10 300 python bench.py > $O/bench_gxf${v}_$i.json 2> $O/bench_gxf${v}_$i.err || exit $?
echo "gxf=$v $(cut -c1-140 $O/bench_gxf${v}_$i.json)"
done
done
