#!/bin/bash
# why is a captured DCGAN / ResNet step slower than eager?  side-stream fork/join inside the capture
# (TBAMD_WGRAD_STREAM_CAPTURE) and stop-event launches (TBAMD_STOP_EVENTS) toggled
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_29; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
W="timeout -k 10 500 python scripts/bench_workloads.py --workload dcgan --mode native --graph --steps 100 --warmup 10"
$W > $O/g_def.log 2>$O/g_def.err; chk $? g_def; echo "g_def $(v g_def)"
TBAMD_WGRAD_STREAM_CAPTURE=0 $W > $O/g_nocap.log 2>$O/g_nocap.err; chk $? g_nocap; echo "g_nocap $(v g_nocap)"
TBAMD_STOP_EVENTS=0 $W > $O/g_nostop.log 2>$O/g_nostop.err; chk $? g_nostop; echo "g_nostop $(v g_nostop)"
TBAMD_WGRAD_STREAM=0 $W > $O/g_noside.log 2>$O/g_noside.err; chk $? g_noside; echo "g_noside $(v g_noside)"
TBAMD_WGRAD_STREAM_CAPTURE=0 timeout -k 10 300 python bench.py --graph on --steps 20 --warmup 8 > $O/r50g_nocap.log 2>$O/r50g_nocap.err; chk $? r50g_nocap; echo "r50g_nocap $(v r50g_nocap)"
echo final rc=0
