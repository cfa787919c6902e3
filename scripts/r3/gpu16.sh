#!/bin/bash
# stop-event fork: stream tests, host-sync test, R50 A/B (stop events on/off, same box), kernel trace;
# GEMM tile decisions of ViT / DCGAN / VAE / LeNet for the shipped table
set -o pipefail
O=gpurun_out/r3_16; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_r2_correctness.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/on$i.log 2>$O/on$i.err; chk $? on$i; tail -1 $O/on$i.log | cut -c1-150
TBAMD_STOP_EVENTS=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/off$i.log 2>$O/off$i.err; chk $? off$i; tail -1 $O/off$i.log | cut -c1-150
done
TBAMD_GEMM_SAVE=$O/tiles_vit.json timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-150
for w in dcgan vae lenet; do
TBAMD_GEMM_SAVE=$O/tiles_$w.json timeout -k 10 300 python scripts/bench_workloads.py --workload $w > $O/$w.log 2>$O/$w.err; chk $? $w; tail -1 $O/$w.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r50 -- python bench.py --steps 4 --warmup 3 > $O/prof.log 2>&1
chk $? prof
