#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_21; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2 3; do
  b m32_$i --steps 20 --warmup 5
  TBAMD_CONV_ROUTES=$R/profiles/r06_m32/routes_before.json b before_$i --steps 20 --warmup 5
done
