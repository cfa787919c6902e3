#!/bin/bash
# 300 timed steps with per-step event times in order: gradual slowdown (clocks / power) or growth?
# GPU clock / power sampled alongside
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_68; mkdir -p $O; cd $R
( for k in $(seq 1 40); do rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|Power|Temperature \(Sensor junction\)|Temperature \(Sensor memory\)" | tr -s ' ' | head -6 | tr '\n' ' '; echo; sleep 0.5; done > $O/smi.txt ) &
SMI=$!
TBAMD_BENCH_STEPTIMES=1 timeout -k 10 400 python bench.py --steps 300 --warmup 5 > $O/b.json 2> $O/b.err; rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
[ $rc -eq 0 ] || exit $rc
python3 - $O <<'PY'
import sys, re
O = sys.argv[1]
t = open(O + "/b.err").read()
m = re.search(r"in order ([0-9. ]+);(.*)", t)
seq = [float(v) for v in m.group(1).split()]
for a in range(0, len(seq), 25):
    chunk = seq[a:a + 25]
    print(f"steps {a:3d}-{a + len(chunk) - 1:3d}: mean {sum(chunk) / len(chunk):.3f} ms")
print(m.group(2).strip())
PY
head -3 $O/smi.txt; tail -3 $O/smi.txt
