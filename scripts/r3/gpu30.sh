#!/bin/bash
# side-stream race fix (fresh-tensor wgrad routes land in the slot on the side stream): stream +
# DDP tests, then the full GPU suite
set -o pipefail
O=gpurun_out/r3_30; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_ddp.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1 ; chk $? pytest; tail -2 $O/pytest.err
