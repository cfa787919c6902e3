#!/bin/bash
# attention forward: scale folded into the exponent fma (one VALU op per score fewer)
# A/B over masks, kernel stats of the default
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_42; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py --model vit_b_16 > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_attention.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for m in 13; do run m${m}_$i TBAMD_ATTN_HEAD=$m; done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o vit -- python3 $R/bench.py --model vit_b_16 --steps 4 --warmup 3 > $O/tr.err 2>&1 || { echo "trace failed"; tail -5 $O/tr.err; exit 1; }
grep -h "attn_" $(find $O/tr -name '*kernel_stats.csv') | cut -d, -f1-4 > $O/attn_stats.txt; cat $O/attn_stats.txt
echo final rc=0
