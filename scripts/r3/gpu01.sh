#!/bin/bash
# round 3, first GPU pass: gpu tests, headline bench, nativized stock ResNet-50,
# self-spawned 2-rank gloo rehearsal, DDP overhead and an RCCL/compute overlap trace
set -o pipefail
O=gpurun_out/r3_01; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1 ; chk $? pytest; tail -2 $O/pytest.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/r50.log 2>$O/r50.err
chk $? r50; tail -1 $O/r50.log | cut -c1-220
timeout -k 10 300 python bench.py --ddp --steps 20 --warmup 5 > $O/r50_ddp1.log 2>$O/r50_ddp1.err
chk $? r50_ddp1; tail -1 $O/r50_ddp1.log | cut -c1-220; grep "ddp buckets" $O/r50_ddp1.err
timeout -k 10 300 python bench.py --model stock_resnet50 --steps 20 --warmup 5 > $O/stock_r50.log 2>$O/stock_r50.err
chk $? stock_r50; tail -1 $O/stock_r50.log | cut -c1-220
TBAMD_BENCH_BACKEND=gloo TBAMD_DDP_CHECK=1 timeout -k 10 300 python bench.py --gpus 2 --batch 32 --steps 3 --warmup 2 > $O/spawn2.log 2>$O/spawn2.err
chk $? spawn2; tail -1 $O/spawn2.log | cut -c1-220
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ddp -o ddp -- python bench.py --steps 4 --warmup 3 --ddp > $O/prof_ddp.log 2>&1
chk $? prof_ddp
python scripts/overlap.py $(ls $O/prof_ddp/*/ddp_kernel_trace.csv $O/prof_ddp/ddp_kernel_trace.csv 2>/dev/null | head -1) > $O/overlap.txt 2>&1; tail -5 $O/overlap.txt
