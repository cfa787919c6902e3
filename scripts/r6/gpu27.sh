#!/bin/bash
# big-tile weight gradient: numerics, per-shape timing, whole-step A/B (interleaved)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_27; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wgrad_big.py > $O/test.log 2>&1; rc=$?; tail -12 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tools/wgrad_big_ab.py > $O/per_shape.txt 2>&1 || exit $?
cat $O/per_shape.txt
for r in 1 2; do
  for v in 0 1; do
    TBAMD_WGRAD_BIG=$v timeout -k 10 300 python bench.py --steps 30 --warmup 8 > $O/bench_big${v}_r$r.json 2> $O/bench_big${v}_r$r.err || exit $?
    echo "big=$v round $r: $(python -c "import json;d=json.load(open('$O/bench_big${v}_r$r.json'));print(d['value'],d['ms_per_step'])")"
  done
done
