#!/bin/bash
# last sanity on the final tree: smoke, headline bench, ViT-S (new tiles), GEMM / conv GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_37; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; chk $? smoke; tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/r50.log 2>$O/r50.err; chk $? r50; echo "r50 $(v r50)"
timeout -k 10 300 python bench.py --model vit_s_16 --batch 128 --steps 15 --warmup 6 > $O/vits.log 2>$O/vits.err; chk $? vits; echo "vits $(v vits)"
timeout -k 10 400 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_gemm*.py tests/test_gpu_tinyin_wgrad.py tests/test_gpu_xf.py > $O/t.err 2>&1; rc=$?; echo "t rc=$rc"; tail -1 $O/t.err
echo final rc=0
