#!/bin/bash
# whole-step kernel trace + PMC passes of the headline ResNet-50 step (one counter group per run);
# BENCH_ARGS="--model vit_b_16 --batch 128" profiles another bench.py config
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${PROF_OUT:-prof}; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o r50 -- python3 $R/bench.py ${BENCH_ARGS} --steps 4 --warmup 3 > $O/tr.err 2>&1; chk $? tr
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py ${BENCH_ARGS} --steps 2 --warmup 3 > $O/pmc_sq.err 2>&1; chk $? pmc_sq
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py ${BENCH_ARGS} --steps 2 --warmup 3 > $O/pmc_fetch.err 2>&1; chk $? pmc_fetch
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py ${BENCH_ARGS} --steps 2 --warmup 3 > $O/pmc_write.err 2>&1; chk $? pmc_write
cd $R
python3 scripts/steady.py $(find $O/tr -name '*kernel_trace.csv' | head -1) 3 1 60 > $O/steady.txt
python3 scripts/pmc_summary.py $O > $O/pmc_summary.txt 2>&1 || true
echo final rc=0
