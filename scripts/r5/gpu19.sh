#!/bin/bash
# whole-head attention forward: tests, then ViT A/B (TBAMD_ATTN_HEAD=0) and a kernel trace of both
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_19; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $O/t.log 2>$O/t.err; rc=$?; tail -3 $O/t.log; chk $rc t
for i in 1 2; do
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/head_$i.log 2>$O/head_$i.err; chk $? head_$i; echo "head_$i $(v head_$i)"
TBAMD_ATTN_HEAD=0 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 > $O/two_$i.log 2>$O/two_$i.err; chk $? two_$i; echo "two_$i $(v two_$i)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/tr.err 2>&1; chk $? tr
cd $R
grep -h "attn" $(find $O/tr -name '*kernel_stats.csv' | head -1) | cut -c1-160
echo final rc=0
