#!/bin/bash
# TN gemm8 split-major XCD mapping: GEMM numerics, ViT-B/16 step A/B (b128 and b256), TN kernel stats + FETCH
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_35; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; b=$2; shift 2; env "$@" timeout -k 10 300 python bench.py --model vit_b_16 --batch $b > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_gemm8.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
run sm128_$i 128 TBAMD_X=0
run old128_$i 128 TBAMD_GEMM8_TN_SPLITMAJOR=0
done
run sm256_1 256 TBAMD_X=0
run old256_1 256 TBAMD_GEMM8_TN_SPLITMAJOR=0
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
TBAMD_GEMM8_TN_SPLITMAJOR=$m timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pf$m -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 2 --warmup 3 > $O/pf$m.err 2>&1 || { echo "pmc $m failed"; tail -5 $O/pf$m.err; exit 1; }
done
echo final rc=0
