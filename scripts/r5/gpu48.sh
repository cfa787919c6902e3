#!/bin/bash
# the shipped route table with ONLY the 8 rows the r5_47 tuning moved to the single-stage big-tile
# kernel (scripts/r5/routes_s1_only.json) vs the shipped table: step A/B, 3 rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_48; mkdir -p $O
chk() { rc=$1; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2 3; do
TBAMD_CONV_ROUTES=$R/scripts/r5/routes_s1_only.json timeout -k 10 300 python bench.py > $O/s1_$i.log 2>$O/s1_$i.err; chk $? s1_$i; echo "s1_$i $(v s1_$i)"
timeout -k 10 300 python bench.py > $O/old_$i.log 2>$O/old_$i.err; chk $? old_$i; echo "old_$i $(v old_$i)"
done
echo final rc=0
