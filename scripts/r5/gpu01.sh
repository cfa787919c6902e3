#!/bin/bash
# round-5 opening: headline bench, whole-step kernel trace (steady-state table), ViT bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_01; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python bench.py > $O/r50.log 2>$O/r50.err; chk $? r50; echo "r50 $(v r50)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_r50 -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr_r50.err 2>&1; chk $? tr_r50
cd $R
f=$(find $O/tr_r50 -name '*kernel_trace.csv' | head -1); python3 scripts/steady.py $f 3 1 80 > $O/r50_steady.txt; head -5 $O/r50_steady.txt
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/vit.log 2>$O/vit.err; chk $? vit; echo "vit $(v vit)"
echo final rc=0
