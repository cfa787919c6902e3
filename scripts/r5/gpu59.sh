#!/bin/bash
# BN finalize slicing 32 / 128 as the default (profiles/r05_colsum): full GPU suite, step A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_${RUN:-59}; mkdir -p $O
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
run() { name=$1; shift; env "$@" timeout -k 10 300 python bench.py > $O/$name.log 2>$O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }; echo "$name $(v $name)"; }
timeout -k 10 1000 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest.err | head -30; tail -2 $O/pytest.err
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
run new_$i TBAMD_X=0
run old_$i TBAMD_COLSUM=64,64
done
echo final rc=0
