#!/bin/bash
# call sites of library-backed ATen ops left in the steady-state steps of the workloads
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_26; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python scripts/r4/aten_calls.py dcgan > $O/dcgan.log 2>$O/dcgan.err; chk $? dcgan; tail -25 $O/dcgan.log
timeout -k 10 300 python scripts/r4/aten_calls.py online --batch 8 --size 256 > $O/online.log 2>$O/online.err; chk $? online; tail -25 $O/online.log
timeout -k 10 300 python scripts/r4/aten_calls.py adain --batch 32 --size 256 > $O/adain.log 2>$O/adain.err; chk $? adain; tail -25 $O/adain.log
echo final rc=0
