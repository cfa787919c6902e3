#!/bin/bash
# streaming bandwidth ceilings (copy / add / sum on a stage-1-sized tensor)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_21; mkdir -p $O
timeout -k 10 120 python scripts/r4/membw.py > $O/membw.log 2>$O/membw.err; rc=$?; echo "membw rc=$rc"; cat $O/membw.log
[ $rc -eq 0 ] || exit $rc
echo final rc=0
