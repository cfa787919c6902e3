#!/bin/bash
# full GPU suite on the current tree (continues past the DDP test) + smoke
set -o pipefail
O=gpurun_out/r3_31; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1 ; chk $? pytest; tail -3 $O/pytest.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.err 2>&1; chk $? smoke; tail -1 $O/smoke.err
