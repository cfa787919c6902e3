#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_04; mkdir -p $O
TBAMD_CONV_NO_MIOPEN=1 timeout -k 10 300 python -u scripts/r5/diag_big.py 64 > $O/diag_nomio.txt 2>&1; echo "diag rc=$?"; head -62 $O/diag_nomio.txt
