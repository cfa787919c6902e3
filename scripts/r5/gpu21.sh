#!/bin/bash
# colsum_fin4 shuffle reduction: BN / conv-stats tests, bench x2, trace (colsum per-call times) + PMC (LDS conflicts)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_21; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_conv1x1p.py tests/test_gpu_xf.py tests/test_gpu_r2_correctness.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; chk $rc t
for i in 1 2; do timeout -k 10 300 python bench.py > $O/b_$i.log 2>$O/b_$i.err; chk $? b_$i; echo "b_$i $(v b_$i)"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr.err 2>&1; chk $? tr
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o r50 -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc.err 2>&1; chk $? pmc
cd $R
T=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/tools/critpath.py $T 3 colsum_fin4 > $O/critpath.txt; sed -n 1,8p $O/critpath.txt; grep "colsum_fin4:" $O/critpath.txt
python3 scripts/r5/pmc_kernels.py $(find $O/pmc -name '*counter_collection.csv' | head -1) colsum > $O/pmc_colsum.txt; cat $O/pmc_colsum.txt
echo final rc=0
