#!/bin/bash
# DCGAN steady state: route timings / ATen library calls, then the kernel census again
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_27; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/r4/aten_calls.py dcgan > $O/dcgan.log 2>$O/dcgan.err; chk $? dcgan; tail -25 $O/dcgan.log; grep -c "tune\]" $O/dcgan.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --mode native --steps 20 --warmup 10 > $O/tr.err 2>&1; chk $? tr
python3 - $(find $O/tr -name '*kernel_trace.csv') > $O/census.txt <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = len(rows); tail = rows[n // 2:]  # second half of the run: steady state
c = collections.Counter(r["Kernel_Name"][:110] for r in tail)
for k, v in c.most_common():
    if any(s in k for s in ("ck::", "igemm", "Cijk", "naive_conv", "miopen", "MIOpen", "SubTensor")):
        print(v, k)
print("total dispatches in window", len(tail))
PY
cat $O/census.txt | head -20
find $O/tr -name '*.csv' -size +20M -delete
echo final rc=0
