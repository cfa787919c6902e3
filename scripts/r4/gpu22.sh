#!/bin/bash
# DCGAN steady-state kernel census (vendor kernels left after the warmup's route tuning), with the
# route decisions logged
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_22; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
cd /tmp && export TMPDIR=/tmp
TBAMD_TUNE_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --mode native --steps 20 --warmup 10 > $O/tr.err 2>&1; chk $? tr
python3 $R/scripts/r4/qsplit.py $(find $O/tr -name '*kernel_trace.csv') --marker adamw_mt_k --last 4 --top 60 > $O/dcgan_qsplit.txt; head -70 $O/dcgan_qsplit.txt
grep -E "conv-tune|gemm-tune" $O/tr.err | cut -c1-220 > $O/tune_log.txt; wc -l $O/tune_log.txt; grep -i miopen $O/tune_log.txt | head -20
find $O/tr -name '*.csv' -size +20M -delete
echo final rc=0
