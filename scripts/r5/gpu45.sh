#!/bin/bash
# BiasSumLink: LayerNorm-backward dx column sums as the residual branch's bias gradient.
# numerics (layernorm, link, attention, trajectory-free ViT tests), ViT-B/16 step A/B b128 / b256
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_45; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; b=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --model vit_b_16 --batch $b > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_layernorm.py tests/test_gpu_bias_link.py tests/test_gpu_attention.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || { tail -30 $O/t.log; exit $rc; }
for i in 1 2; do
run link128_$i 128 TBAMD_X=0
run off128_$i 128 TBAMD_BIAS_SUM_LINK=0
done
run link256_1 256 TBAMD_X=0
run off256_1 256 TBAMD_BIAS_SUM_LINK=0
echo final rc=0
