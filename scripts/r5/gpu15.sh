#!/bin/bash
# ViT-B/16 b128 (current defaults: hipBLASLt candidate on): steady kernel table + PMC (MFMA busy) per kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_15; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/tr.err 2>&1; chk $? tr
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 2 --warmup 3 > $O/pmc.err 2>&1; chk $? pmc
cd $R
T=$(find $O/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/steady.py $T 3 1 40 > $O/steady.txt
P=$(find $O/pmc -name '*counter_collection.csv' | head -1)
python3 scripts/r5/pmc_kernels.py $P > $O/pmc_table.txt
head -25 $O/steady.txt; head -25 $O/pmc_table.txt
echo final rc=0
