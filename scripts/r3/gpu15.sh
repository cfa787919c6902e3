#!/bin/bash
# fork cost variants (native), nativized stock ResNet-50 with the side stream, ViT-B/16 kernel trace
set -o pipefail
O=gpurun_out/r3_15; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 60 scripts/r3/native/fork_cost > $O/fork.log 2>$O/fork.err; chk $? fork; cat $O/fork.log
timeout -k 10 300 python bench.py --model stock_resnet50 --steps 30 --warmup 10 > $O/st50.log 2>$O/st50.err
chk $? st50; tail -1 $O/st50.log | cut -c1-200
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err
chk $? vit; tail -1 $O/vit.log | cut -c1-200; grep -c gemm-tune $O/vit.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o vit -- python bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/prof.log 2>&1
chk $? prof
