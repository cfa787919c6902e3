#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_13; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_memory.py tests/test_gpu_res_carrier.py > $O/tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|retained" $O/tests.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tools/leak_probe.py > $O/leak.txt 2> $O/leak.err || exit $?; head -6 $O/leak.txt
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2; do
  b new_$i --steps 20 --warmup 5
  TBAMD_COLSUM_SCALAR=1 b scalar_$i --steps 20 --warmup 5
done
timeout -k 10 400 python scripts/tools/lmdb_e2e.py > $O/lmdb.json 2> $O/lmdb.err; rc=$?; cat $O/lmdb.json; exit $rc
