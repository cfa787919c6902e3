#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_04; mkdir -p $O
timeout -k 10 300 python -u scripts/r4/nondet_fwd.py > $O/nf.log 2>&1; echo "r18 rc=$?"; tail -3 $O/nf.log
TBAMD_COLSUM=1000000,1 timeout -k 10 300 python -u scripts/r4/nondet_fwd.py > $O/nf1.log 2>&1; echo "single-slice rc=$?"; tail -3 $O/nf1.log
MODEL=resnet50 timeout -k 10 300 python -u scripts/r4/nondet_fwd.py > $O/nf50.log 2>&1; echo "r50 rc=$?"; tail -3 $O/nf50.log
