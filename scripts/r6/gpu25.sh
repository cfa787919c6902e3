#!/bin/bash
# lazy-BN running-stats probe; the rest of the GPU suite after test_gpu_xf; smoke(); default bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_25; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/tools/xf_buffer_probe.py > $O/probe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_xf.py tests/test_graph_step.py tests/test_models.py tests/test_native_host.py tests/test_nativize.py tests/test_scheduler.py tests/test_trace.py tests/test_tune_agree.py tests/test_utils.py -rf > $O/rest.log 2>&1; rc=$?; tail -3 $O/rest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cat $O/bench_default.json
