#!/bin/bash
# gemm8 with scalar-base staging: tests + bench + PMC
set -o pipefail
O=gpurun_out/r3_05; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm8.py > $O/t.err 2>&1 ; chk $? t; tail -1 $O/t.err
timeout -k 10 300 python -u scripts/gemm8_bench.py > $O/gemm8_bench.log 2>$O/gemm8_bench.err
chk $? gemm8_bench; python3 -c "
import json
for l in open('$O/gemm8_bench.log'):
    d=json.loads(l); print(d['shape'], 'blas', d['blas_tf'], 't16', d['t16_tf'], 't16ns', d['t16ns_tf'], 't0', d['t0_tf'], 't1', d['t1_tf'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p1 -o p1 -- python3 scripts/r3/gemm_pmc.py > $O/p1.log 2>&1
echo "p1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o p2 -- python3 scripts/r3/gemm_pmc.py > $O/p2.log 2>&1
echo "p2 rc=$?"
python3 scripts/r3/pmc_by_kernel.py $(find $O/p1 -name "*counter_collection.csv") | grep -v "at::native\|rocclr\|Functor"
python3 scripts/r3/pmc_by_kernel.py $(find $O/p2 -name "*counter_collection.csv") | grep -v "at::native\|rocclr\|Functor"
