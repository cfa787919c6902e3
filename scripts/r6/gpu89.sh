#!/bin/bash
# ViT-B/16 b128 kernel trace, --ddp (1-rank RCCL) vs plain: where the 3.7 % goes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_89; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ddp -o r50 -- python3 $R/bench.py --model vit_b_16 --batch 128 --ddp --steps 4 --warmup 4 > $O/ddp.out 2> $O/ddp.err || { tail -20 $O/ddp.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/plain -o r50 -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 4 > $O/plain.out 2> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
cd $R
python3 scripts/steady.py $(find $O/ddp -name '*kernel_trace.csv' | head -1) 3 1 80 > $O/steady_ddp.txt
python3 scripts/steady.py $(find $O/plain -name '*kernel_trace.csv' | head -1) 3 1 80 > $O/steady_plain.txt
head -1 $O/steady_ddp.txt; head -1 $O/steady_plain.txt
