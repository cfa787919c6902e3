#!/bin/bash
# host-boundness of the ResNet-50 step: host submit time, event-fork gap cost, graph replay with
# the wgrad side stream captured; plus the GPU tests that -x stopped before in r3_13
set -o pipefail
O=gpurun_out/r3_14; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 120 python scripts/r3/event_gap.py > $O/ev.log 2>$O/ev.err; chk $? ev; cat $O/ev.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/r50.log 2>$O/r50.err
chk $? r50; tail -1 $O/r50.log | cut -c1-200; grep "host submit" $O/r50.err
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --graph on > $O/r50g.log 2>$O/r50g.err
chk $? r50g; tail -1 $O/r50g.log | cut -c1-200; grep "host submit" $O/r50g.err
TBAMD_WGRAD_STREAM_CAPTURE=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 --graph on > $O/r50g0.log 2>$O/r50g0.err
chk $? r50g0; tail -1 $O/r50g0.log | cut -c1-200
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_r2_correctness.py tests/test_gpu_s* tests/test_gpu_t* > $O/pytest.err 2>&1 ; chk $? pytest; tail -2 $O/pytest.err
