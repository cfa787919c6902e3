#!/bin/bash
# host-side (Python) profile of the headline step: the host submits at ~90 % of the GPU time
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_32; mkdir -p $O; cd $R
timeout -k 10 300 python -m cProfile -o $O/bench.pstats bench.py --steps 30 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-150 $O/bench.json; grep "host submit" $O/bench.err
python - <<'PY' > $O/pstats_top.txt
import pstats, os
p = pstats.Stats(os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r6_32/bench.pstats")
p.sort_stats("tottime").print_stats(60)
p.sort_stats("cumulative").print_stats(80)
PY
head -120 $O/pstats_top.txt
