#!/bin/bash
# BN finalize slicing (TBAMD_COLSUM=min_rows,max_slices) re-checked on the 16384-cap tree, alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_53; mkdir -p $O; cd $R
for i in 1 2; do
for c in 32,128 16,256 32,256 64,64; do
TBAMD_COLSUM=$c timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "colsum=$c $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
