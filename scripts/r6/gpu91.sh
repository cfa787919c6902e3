#!/bin/bash
# last closing check (late-init side-stream replacement in): bitwise BN test, full GPU suite, smoke, bench x2, ViT-B/16
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_91; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_bn_grid.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1; rc=$?
tail -2 $O/gpu_suite.log; grep -E "^(FAILED|ERROR)" $O/gpu_suite.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
echo "r50 $(python3 -c "import json;d=json.load(open('$O/bench_$i.json'));print(d['value'],d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/vit.json 2> $O/vit.err || exit $?
echo "vit $(python3 -c "import json;d=json.load(open('$O/vit.json'));print(d['value'],d['ms_per_step'])")"
