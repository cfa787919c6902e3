#!/bin/bash
# ResNet-50 b256 steady-state kernel trace + main-stream critical path
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_08; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr.err 2>&1 || { tail -20 $O/tr.err; exit 1; }
cd $R
T=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/steady.py $T 3 1 60 > $O/steady.txt
python3 scripts/tools/critpath.py $T 3 > $O/critpath.txt 2>&1
head -30 $O/critpath.txt
