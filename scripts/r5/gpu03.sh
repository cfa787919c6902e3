#!/bin/bash
# PMC of the big-tile conv vs the 128x128 kernel on three 3x3 forward shapes; fixed tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_03; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_gpu_conv_big.py -k heuristic tests/test_gpu_f32_exact.py > $O/t.err 2>&1; echo "t rc=$?"; grep -E "deviation|exact|passed|failed" $O/t.err | tail -12
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o run -- python3 $R/scripts/r5/conv_big_bench.py --only 128:28:128:3:1,256:14:256:3:1,64:56:64:3:1 --kinds fwd --rounds 1 --iters 3 --check 0 --codes "128,256,16,3;256,256,16,2;128,128,16,4" > $O/pmc.err 2>&1; chk $? pmc
cd $R
python3 scripts/r5/pmc_kernels.py $(find $O/pmc -name '*counter_collection.csv' | head -1) conv > $O/pmc_table.txt; cat $O/pmc_table.txt
echo final rc=0
