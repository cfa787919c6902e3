#!/bin/bash
# fused max-pool + BN backward (stem) and colsum slice sizing: tests, then whole-step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_11; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "maxpool or bn_" > $O/t.log 2>$O/t.err; rc=$?; tail -3 $O/t.log; chk $rc t
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/fused_$i.log 2>$O/fused_$i.err; chk $? fused_$i; echo "fused_$i $(v fused_$i)"
TBAMD_POOL_FUSED_BWD=0 timeout -k 10 300 python bench.py > $O/unf_$i.log 2>$O/unf_$i.err; chk $? unf_$i; echo "unf_$i $(v unf_$i)"
done
echo final rc=0
