#!/bin/bash
# kernel trace of the --ddp (1-rank RCCL) step vs the plain step on one box: which kernels / gaps add 2.5 ms
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_84; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ddp -o r50 -- python3 $R/bench.py --ddp --steps 4 --warmup 3 > $O/ddp.out 2> $O/ddp.err || { tail -20 $O/ddp.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/plain -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/plain.out 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
cd $R
python3 scripts/steady.py $(find $O/ddp -name '*kernel_trace.csv' | head -1) 3 1 80 > $O/steady_ddp.txt
python3 scripts/steady.py $(find $O/plain -name '*kernel_trace.csv' | head -1) 3 1 80 > $O/steady_plain.txt
head -1 $O/steady_ddp.txt; head -1 $O/steady_plain.txt
