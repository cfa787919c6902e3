#!/bin/bash
# full GPU suite on the round-6 tree; reverse-XF upper bound diagnostic; LMDB -> prefetcher re-measure
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_10; mkdir -p $O; cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2; do
  b base_$i --steps 20 --warmup 5
  TBAMD_DIAG_SKIP_BN_BWD=inner b skip_inner_$i --steps 20 --warmup 5
  TBAMD_DIAG_SKIP_BN_BWD=all b skip_all_$i --steps 20 --warmup 5
done
timeout -k 10 400 python scripts/tools/lmdb_e2e.py > $O/lmdb.json 2> $O/lmdb.err; rc=$?; cat $O/lmdb.json; exit $rc
