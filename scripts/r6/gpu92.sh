#!/bin/bash
# plain N=1 step: side stream at the caller's priority (auto without a group) vs low priority, alternated 4x
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_92; mkdir -p $O; cd $R
for i in 1 2 3 4; do
for v in auto low; do
TBAMD_SIDE_PRIORITY=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "side=$v r50 $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
