#!/bin/bash
# BN streaming passes: total workgroups of the apply kernels (TBAMD_BN_APPLY_WG, min row passes per
# workgroup TBAMD_BN_APPLY_MINPASS) -- the probe (r6_36) streams 6.0 TB/s with one 16-B vector per
# thread over a full grid and 5.1 TB/s with 2048 long-lived chunked workgroups; step A/B alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_37; mkdir -p $O; cd $R
for i in 1 2; do
for cfg in 2048:2 8192:2 32768:2 131072:2 131072:1; do
wg=${cfg%:*}; mp=${cfg#*:}
TBAMD_BN_APPLY_WG=$wg TBAMD_BN_APPLY_MINPASS=$mp timeout -k 10 300 python bench.py --steps 30 > $O/b_${wg}_${mp}_$i.json 2> $O/b_${wg}_${mp}_$i.err || exit $?
echo "wg=$wg minpass=$mp $(python3 -c "import json;d=json.load(open('$O/b_${wg}_${mp}_$i.json'));print(d['value'],d['ms_per_step'])")"
done
done
