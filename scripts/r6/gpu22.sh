#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_22; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gelu_link.py tests/test_gpu_linear.py > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2 3; do
  b nt_$i --model vit_b_16 --batch 128 --steps 20 --warmup 5
  TBAMD_GELU_BWD_NT=0 b nn_$i --model vit_b_16 --batch 128 --steps 20 --warmup 5
done
