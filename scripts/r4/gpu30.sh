#!/bin/bash
# style-transfer steps eager vs captured (now that captures stay on one stream)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_30; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
W="timeout -k 10 400 python scripts/bench_workloads.py --steps 40 --warmup 8"
for g in "" "--graph"; do
t=${g:+g}
$W --workload online --batch 8 --size 256 --mode native $g > $O/online$t.log 2>$O/online$t.err; chk $? online$t; echo "online$t $(v online$t)"
$W --workload online --batch 8 --size 256 --mode native32 $g > $O/online32$t.log 2>$O/online32$t.err; chk $? online32$t; echo "online32$t $(v online32$t)"
$W --workload adain --batch 32 --size 256 --mode native $g > $O/adain$t.log 2>$O/adain$t.err; chk $? adain$t; echo "adain$t $(v adain$t)"
$W --workload nst --batch 1 --size 512 --mode native32 $g > $O/nst32$t.log 2>$O/nst32$t.err; chk $? nst32$t; echo "nst32$t $(v nst32$t)"
done
echo final rc=0
