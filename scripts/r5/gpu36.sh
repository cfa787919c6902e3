#!/bin/bash
# 1x1 weight gradients on the TN GEMM (gemm8 TN, split-major) instead of conv_wgrad_k: step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_36; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
for i in 1 2; do
run base_$i TBAMD_X=0
run gemm_$i TBAMD_CONV_WGRAD=gemm
done
cd /tmp && export TMPDIR=/tmp
TBAMD_CONV_WGRAD=gemm timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr.err 2>&1 || { echo "trace failed"; tail -5 $O/tr.err; exit 1; }
cd $R && python3 scripts/steady.py $(find $O/tr -name '*kernel_trace.csv' | head -1) 3 1 40 > $O/steady.txt && head -25 $O/steady.txt
echo final rc=0
