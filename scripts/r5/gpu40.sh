#!/bin/bash
# per-shape weight-gradient traffic (FETCH_SIZE / WRITE_SIZE) of every ResNet-50 b256 weight gradient run alone
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_40; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pf -o run -- python3 $R/scripts/r5/wgrad_bytes.py > $O/pf.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/pf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pw -o run -- python3 $R/scripts/r5/wgrad_bytes.py > $O/pw.log 2>&1 || { echo "write pass failed"; tail -5 $O/pw.log; exit 1; }
echo final rc=0
