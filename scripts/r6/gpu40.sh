#!/bin/bash
# downsample-partials BN apply and stem pool partial grids (TBAMD_BN_DSP_WG / TBAMD_BN_POOL_WG), step A/B alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_40; mkdir -p $O; cd $R
for i in 1 2; do
for cfg in 2048:2048 8192:2048 16384:2048 2048:8192; do
d=${cfg%:*}; p=${cfg#*:}
TBAMD_BN_DSP_WG=$d TBAMD_BN_POOL_WG=$p timeout -k 10 300 python bench.py --steps 30 > $O/b_${d}_${p}_$i.json 2> $O/b_${d}_${p}_$i.err || exit $?
echo "dsp=$d pool=$p $(python3 -c "import json;d=json.load(open('$O/b_${d}_${p}_$i.json'));print(d['value'],d['ms_per_step'])")"
done
done
