#!/bin/bash
# big-tile conv: numerics, per-shape A/B vs the 128x128 kernels, whole-step A/B; stream/one-shot changes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_02; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_gpu_conv_big.py > $O/t_big.err 2>&1; echo "t_big rc=$?"; grep -E "worst parameter|passed|failed" $O/t_big.err | tail -4
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_oneshot.py tests/test_gpu_f32_exact.py > $O/t_str.err 2>&1; echo "t_str rc=$?"; tail -3 $O/t_str.err
timeout -k 10 500 python -u scripts/r5/conv_big_bench.py --rounds 3 --iters 4 > $O/ab.jsonl 2>$O/ab.err; chk $? ab
for i in 1 2; do
TBAMD_CONV_BIG=1 timeout -k 10 300 python bench.py > $O/big_$i.log 2>$O/big_$i.err; chk $? big_$i; echo "big_$i $(v big_$i)"
timeout -k 10 300 python bench.py > $O/old_$i.log 2>$O/old_$i.err; chk $? old_$i; echo "old_$i $(v old_$i)"
done
TBAMD_BENCH_HIPRI=1 timeout -k 10 300 python bench.py > $O/hipri.log 2>$O/hipri.err; chk $? hipri; echo "hipri $(v hipri)"
echo final rc=0
