#!/bin/bash
# BiasSumLink on/off (DXS LayerNorm backward without prefetch, 2 waves/SIMD): step A/B + kernel stats of the ViT-B/16 b128 step (LayerNorm backward, column sums)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_46; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; b=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --model vit_b_16 --batch $b > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_layernorm.py tests/test_gpu_bias_link.py > $O/t.log 2>$O/t.err; rc=$?; tail -1 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
run link128_$i 128 TBAMD_X=0
run off128_$i 128 TBAMD_BIAS_SUM_LINK=0
run link256_$i 256 TBAMD_X=0
run off256_$i 256 TBAMD_BIAS_SUM_LINK=0
done
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
TBAMD_BIAS_SUM_LINK=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$m -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 6 --warmup 3 > $O/tr$m.err 2>&1 || { echo "trace $m failed"; tail -5 $O/tr$m.err; exit 1; }
grep -h "ln_bwd\|col_sum\|colsum\|convert\|copy" $(find $O/tr$m -name '*kernel_stats.csv') | cut -d, -f1-4 | cut -c1-160 > $O/stats_$m.txt; echo "== $m"; cat $O/stats_$m.txt
done
echo final rc=0
