#!/bin/bash
# downsample-BN partials from the block-output BN's backward apply (TBAMD_DS_PARTIALS): numerics,
# step A/B, kernel time
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_57; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_res_carrier.py tests/test_gpu_xf.py tests/test_gpu_trajectory.py > $O/t.log 2>$O/t.err; rc=$?; tail -2 $O/t.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $O/t.log | head -20; exit $rc; }
for i in 1 2 3; do
run dsp_$i TBAMD_X=0
run old_$i TBAMD_DS_PARTIALS=0
done
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
TBAMD_DS_PARTIALS=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$m -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr$m.err 2>&1 || { echo "trace $m failed"; tail -5 $O/tr$m.err; exit 1; }
done
echo final rc=0
