#!/bin/bash
# whole-step kernel trace of the headline step: main-stream critical path and colsum per-call times
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_10; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr.err 2>&1; chk $? tr
cd $R
T=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/tools/critpath.py $T 3 colsum_fin4 > $O/critpath.txt && python3 scripts/steady.py $T 3 1 60 > $O/steady.txt
head -60 $O/critpath.txt
gzip -c $T > $O/trace.csv.gz
echo final rc=0
