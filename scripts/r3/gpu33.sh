#!/bin/bash
# ViT-B/16 b128: bench + whole-step kernel trace
set -o pipefail
O=gpurun_out/r3_33; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o vit -- python bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/prof.err 2>&1
chk $? prof
