#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_04; mkdir -p $O
timeout -k 10 300 python -u scripts/r4/nondet.py > $O/nd.log 2>&1; echo "default rc=$?"; tail -9 $O/nd.log
TBAMD_COLSUM=1000000,1 timeout -k 10 300 python -u scripts/r4/nondet.py > $O/nd1.log 2>&1; echo "single-slice rc=$?"; tail -9 $O/nd1.log
TBAMD_COLSUM_WT=0 timeout -k 10 300 python -u scripts/r4/nondet.py > $O/nd2.log 2>&1; echo "release-fence rc=$?"; tail -9 $O/nd2.log
