#!/bin/bash
# ViT-B/16 regression since round 2: HEAD vs HEAD+hipBLASLt vs HEAD with the round-4 stream setup vs
# the round-2 tree, then a kernel trace of each tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_06; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
VB="bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8"
timeout -k 10 300 python $VB > $O/head.log 2>$O/head.err; chk $? head; echo "head $(v head)"
TBAMD_GEMM_BLAS=1 timeout -k 10 300 python $VB > $O/blas.log 2>$O/blas.err; chk $? blas; echo "blas $(v blas)"
TBAMD_SIDE_PRIORITY=normal TBAMD_BENCH_HIPRI=1 timeout -k 10 300 python $VB > $O/r4str.log 2>$O/r4str.err; chk $? r4str; echo "r4str $(v r4str)"
(cd .bisect/r2 && timeout -k 10 300 python $VB) > $O/r2.log 2>$O/r2.err; chk $? r2; echo "r2 $(v r2)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_head -o t -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/tr_head.err 2>&1; chk $? tr_head
cd $R/.bisect/r2
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_r2 -o t -- python3 $R/.bisect/r2/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/tr_r2.err 2>&1; chk $? tr_r2
cd $R
for t in head r2; do python3 scripts/steady.py $(find $O/tr_$t -name '*kernel_trace.csv' | head -1) 3 1 40 > $O/steady_$t.txt; head -3 $O/steady_$t.txt; done
echo final rc=0
