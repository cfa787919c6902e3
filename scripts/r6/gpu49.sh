#!/bin/bash
# BN apply grid: old / full / 4-row / capped on ResNet-50 and ResNet-101, alternated twice
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_49; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; }
for i in 1 2; do
for cfg in 2048:2 131072:2 131072:4 16384:2; do
wg=${cfg%:*}; mp=${cfg#*:}
TBAMD_BN_APPLY_WG=$wg TBAMD_BN_APPLY_MINPASS=$mp b r50 python bench.py --steps 20
TBAMD_BN_APPLY_WG=$wg TBAMD_BN_APPLY_MINPASS=$mp b r101 python bench.py --model resnet101 --steps 20
echo "wg=$wg mp=$mp r50 $(python3 -c "import json;d=json.load(open('$O/r50.json'));print(d['value'])") r101 $(python3 -c "import json;d=json.load(open('$O/r101.json'));print(d['value'])")"
done
done
