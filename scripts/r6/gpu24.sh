#!/bin/bash
# round-6 tree check: full GPU suite, smoke(), the driver's bench invocation
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_24; mkdir -p $O; cd $R
timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1; rc=$?; tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json | cut -c1-300
