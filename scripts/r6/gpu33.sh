#!/bin/bash
# host-side A/B: Python's cyclic GC during the timed steps (default vs gc.freeze after warmup), with
# per-step event times; alternated on one box
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_33; mkdir -p $O; cd $R
for i in 1 2; do
for v in "" freeze; do
TBAMD_BENCH_STEPTIMES=1 TBAMD_BENCH_GC=$v timeout -k 10 300 python bench.py --steps 40 > $O/b_${v:-default}_$i.json 2> $O/b_${v:-default}_$i.err || exit $?
echo "gc=${v:-default} $(cut -c90-150 $O/b_${v:-default}_$i.json) $(grep 'per-step' $O/b_${v:-default}_$i.err | cut -c1-90)"
grep "host submit" $O/b_${v:-default}_$i.err
done
done
