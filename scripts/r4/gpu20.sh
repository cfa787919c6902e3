#!/bin/bash
# DCGAN eager vs graph: kernel statistics of each (why is the replayed step 2x slower?); the
# BN-in-operand tests after the hook guard
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_20; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_xf.py > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed" $O/t.err | tail -2
cd /tmp && export TMPDIR=/tmp
for m in eager graph; do
  g=""; [ $m = graph ] && g="--graph"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$m -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --mode native --steps 30 --warmup 10 $g > $O/tr_$m.err 2>&1; chk $? tr_$m
  f=$(find $O/tr_$m -name '*kernel_stats.csv' | head -1)
  python3 - "$f" > $O/stats_$m.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot/1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
for r in rows[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:8.3f} ms {int(r['Calls']):6d}  {r['Name'][:100]}")
PY
  head -27 $O/stats_$m.txt
  find $O/tr_$m -name '*.csv' ! -name '*kernel_stats.csv' -delete
done
echo final rc=0
