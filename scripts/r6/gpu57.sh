#!/bin/bash
# compute stream at high priority (TBAMD_BENCH_HIPRI=1, the round-4 arrangement) re-checked on the closing tree
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_57; mkdir -p $O; cd $R
for i in 1 2 3; do
for v in 0 1; do
TBAMD_BENCH_HIPRI=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "hipri=$v $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
