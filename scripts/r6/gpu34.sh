#!/bin/bash
# full GPU suite + smoke + the driver's bench invocation on the session-2 tree
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_34; mkdir -p $O; cd $R
timeout -k 10 1100 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1; rc=$?
tail -3 $O/gpu_suite.log; grep -E "^(FAILED|ERROR)" $O/gpu_suite.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-200 $O/bench.json
