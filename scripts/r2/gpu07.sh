# PMC: MFMA busy / waits / clock for gemm tile 0 vs ping-pong vs hipBLASLt at 4096^3
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_07
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p1 -o p1 -- python3 scripts/r2/pp_pmc.py > $O/p1.log 2>&1
echo p1 rc=$?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $O/p2 -o p2 -- python3 scripts/r2/pp_pmc.py > $O/p2.log 2>&1
echo p2 rc=$?
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 scripts/r2/pp_pmc.py > $O/kt.log 2>&1
echo kt rc=$?
find $O -name "*.csv" | head
