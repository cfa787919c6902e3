#!/bin/bash
# the full GPU test suite on the current tree + smoke()
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_11; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest.err | head -30; tail -3 $O/pytest.err
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.log
