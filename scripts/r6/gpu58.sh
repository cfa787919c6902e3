#!/bin/bash
# the driver's exact bench invocation on whatever box this call lands on (distribution of the closing tree)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_58; mkdir -p $O; cd $R
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$(date +%s).json 2> $O/bench.err || exit $?
for f in $O/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print(d['value'],d['ms_per_step'])"; done
