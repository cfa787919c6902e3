#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_04; mkdir -p $O
TBAMD_CONV_NO_MIOPEN=1 timeout -k 10 300 python -u scripts/r5/diag_big4.py > $O/diag4.txt 2>&1; echo "diag rc=$?"; grep -v "y-diff 0 aux rows [0-9/]* aux-diff [0-9.e-]*$" $O/diag4.txt | tail -40; grep -c "y-diff" $O/diag4.txt
