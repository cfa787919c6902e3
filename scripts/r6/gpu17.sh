#!/bin/bash
# dS-materialising attention backward: numerics (all mask variants, bounds-checked build too), then ViT A/B
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_17; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_attention.py > $O/tests.log 2>&1; rc=$?; grep -cE "PASSED" $O/tests.log; grep -E "FAIL|Error" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
TBAMD_BOUNDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_attention.py -k "variants" > $O/tests_bounds.log 2>&1; rc=$?; tail -2 $O/tests_bounds.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
for i in 1 2; do
  b ds13_$i --model vit_b_16 --batch 128 --steps 20 --warmup 5
  TBAMD_ATTN_HEAD=5 b old5_$i --model vit_b_16 --batch 128 --steps 20 --warmup 5
done
b ds13_b256 --model vit_b_16 --batch 256 --steps 10 --warmup 4
TBAMD_ATTN_HEAD=5 b old5_b256 --model vit_b_16 --batch 256 --steps 10 --warmup 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o r -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/st.err 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, os
f = glob.glob(os.environ.get("GRAFT_REPO_ROOT") + "/gpurun_out/r6_17/st/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "attn" in r["Name"] or "Cijk" in r["Name"]:
        print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
