#!/bin/bash
# what the round-5 reference cycle (~5 GB/step retained) cost the timed loop: same box, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_15; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2 3; do
  b fixed_$i --steps 20 --warmup 5
  TBAMD_DIAG_STRONGREF=1 b leak_$i --steps 20 --warmup 5
done
TBAMD_DIAG_STRONGREF=1 b leak_long --steps 40 --warmup 5
b fixed_long --steps 40 --warmup 5
