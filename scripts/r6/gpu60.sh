#!/bin/bash
# dgrad-epilogue kernels with a pipelined k-loop (TBAMD_CONV_EPI_STAGES=2|3) re-checked on the closing tree
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_60; mkdir -p $O; cd $R
for i in 1 2; do
for v in 1 2 3; do
TBAMD_CONV_EPI_STAGES=$v timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?
echo "epi_stages=$v $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])")"
done
done
