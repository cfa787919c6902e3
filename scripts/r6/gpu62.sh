#!/bin/bash
# BN finalize: fatter slices (fewer two-phase launches; TBAMD_COLSUM=min_rows,max_slices), alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_62; mkdir -p $O; cd $R
for i in 1 2; do
for c in 32,128 128,128 256,64 64,128; do
TBAMD_COLSUM=$c timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "colsum=$c $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
