#!/bin/bash
# write-through slab publish in the BN finalize reductions (no buffer_wbl2): BN numerics tests,
# 20-step trajectory tests, ResNet-50 A/B alternated (TBAMD_COLSUM_WT=1 default vs 0)
set -o pipefail
O=gpurun_out/r3_22; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_trajectory.py tests/test_gpu_r2_correctness.py tests/test_gpu_streams.py tests/test_gpu_act.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/wt$i.log 2>$O/wt$i.err; chk $? wt$i; tail -1 $O/wt$i.log | cut -c1-120
TBAMD_COLSUM_WT=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/fence$i.log 2>$O/fence$i.err; chk $? fence$i; tail -1 $O/fence$i.log | cut -c1-120
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r50 -- python bench.py --steps 4 --warmup 3 > $O/prof.log 2>&1
chk $? prof
