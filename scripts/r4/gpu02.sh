#!/bin/bash
# ADVICE fixes + framework priority stream + tail bucket: targeted tests, full GPU suite, bench
# plain vs --ddp (alternated), --ddp kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_02; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_shared_weight.py tests/test_gpu_r2_correctness.py tests/test_gpu_streams.py tests/test_gpu_ddp.py > $O/t.err 2>&1; chk $? t; grep -E "passed|failed" $O/t.err | tail -2
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1; chk $? pytest; tail -2 $O/pytest.err
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/plain$i.log 2>$O/plain$i.err; chk $? plain$i; tail -1 $O/plain$i.log | cut -c1-150
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --ddp > $O/ddp$i.log 2>$O/ddp$i.err; chk $? ddp$i; tail -1 $O/ddp$i.log | cut -c1-150
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr_ddp -o ddp -- python3 $R/bench.py --steps 4 --warmup 3 --ddp > $O/tr_ddp.err 2>&1; chk $? tr_ddp
python3 $R/scripts/r4/qsplit.py $(find $O/tr_ddp -name '*kernel_trace.csv') --top 8 > $O/ddp_qsplit.txt; head -50 $O/ddp_qsplit.txt
