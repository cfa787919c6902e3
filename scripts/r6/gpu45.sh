#!/bin/bash
# kernel trace of the closing tree (full-grid BN passes)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_45; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr.err 2>&1 || exit $?
cd $R && python3 scripts/steady.py $(find $O/tr -name '*kernel_trace.csv' | head -1) 3 1 60 > $O/steady.txt && head -25 $O/steady.txt
