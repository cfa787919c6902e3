#!/bin/bash
# PMC passes on gemm8 vs hipBLASLt vs tile 0
set -o pipefail
O=gpurun_out/r3_04; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p1 -o p1 -- python3 scripts/r3/gemm_pmc.py > $O/p1.log 2>&1
echo "p1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 scripts/r3/gemm_pmc.py > $O/p2.log 2>&1
echo "p2 rc=$?"
python3 scripts/r3/pmc_by_kernel.py $(find $O/p1 -name "*counter_collection.csv") > $O/p1.txt; cat $O/p1.txt
python3 scripts/r3/pmc_by_kernel.py $(find $O/p2 -name "*counter_collection.csv") > $O/p2.txt; cat $O/p2.txt
