#!/bin/bash
# deterministic stream/reducer tests + trajectory, 1x1 persistent conv A/B + numerics, benches
# plain vs --ddp, --ddp kernel trace, then the full GPU suite
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_05; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
# test steps: a failing test (rc 1) is reported and the script goes on; a crash / timeout stops it
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_conv1x1p.py > $O/c1.err 2>&1; chkt $? c1; grep -E "passed|failed" $O/c1.err | tail -2
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_bn_fold.py > $O/fold.err 2>&1; chkt $? fold; grep -E "passed|failed" $O/fold.err | tail -2
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_r4_routes.py > $O/rt.err 2>&1; chkt $? rt; grep -E "passed|failed" $O/rt.err | tail -2
timeout -k 10 300 python scripts/r4/routes_bench.py > $O/routes.log 2>$O/routes.err; chk $? routes; cat $O/routes.log
TBAMD_CONV1X1P=0 timeout -k 10 300 python scripts/r4/conv1x1_bench.py > $O/c1x1_off.log 2>$O/c1x1_off.err; chk $? c1x1_off
timeout -k 10 300 python scripts/r4/conv1x1_bench.py > $O/c1x1_on.log 2>$O/c1x1_on.err; chk $? c1x1_on
paste -d' ' <(cut -c1-100 $O/c1x1_off.log) <(cut -c40-100 $O/c1x1_on.log) | head -40
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/plain$i.log 2>$O/plain$i.err; chk $? plain$i; tail -1 $O/plain$i.log | cut -c1-150
TBAMD_BN_FOLD=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/f0$i.log 2>$O/f0$i.err; chk $? f0$i; tail -1 $O/f0$i.log | cut -c1-150
TBAMD_CONV1X1P=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/p0$i.log 2>$O/p0$i.err; chk $? p0$i; tail -1 $O/p0$i.log | cut -c1-150
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --ddp > $O/ddp$i.log 2>$O/ddp$i.err; chk $? ddp$i; tail -1 $O/ddp$i.log | cut -c1-150
done
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_shared_weight.py tests/test_gpu_streams.py tests/test_gpu_ddp.py tests/test_gpu_trajectory.py tests/test_gpu_oneshot.py -s > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed|deviation" $O/t.err | tail -6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr_ddp -o ddp -- python3 $R/bench.py --steps 4 --warmup 3 --ddp > $O/tr_ddp.err 2>&1; chk $? tr_ddp
python3 $R/scripts/r4/qsplit.py $(find $O/tr_ddp -name '*kernel_trace.csv') --top 12 > $O/ddp_qsplit.txt; head -40 $O/ddp_qsplit.txt
cd $R
