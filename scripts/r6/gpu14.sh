#!/bin/bash
# colsum finalize reducer A/B: kernel stats + interleaved whole-step bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_14; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2 3; do
  b new_$i --steps 20 --warmup 5
  TBAMD_COLSUM_RED=0 b old_$i --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_new -o r -- python3 $R/bench.py --steps 5 --warmup 3 > $O/st_new.err 2>&1 || exit 1
TBAMD_COLSUM_RED=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_old -o r -- python3 $R/bench.py --steps 5 --warmup 3 > $O/st_old.err 2>&1 || exit 1
for v in new old; do echo $v; grep -h colsum_fin4 $(find $O/st_$v -name '*kernel_stats.csv') | cut -d, -f1-6; done
