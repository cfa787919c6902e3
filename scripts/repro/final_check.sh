#!/bin/bash
# closing check on the current tree: full GPU suite + smoke, headline bench x2, ViT-B/16, the
# ResNet-50 ImageNet-config example, and the secondary workloads (eager and hipGraph)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${FINAL_OUT:-final}; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 1000 python -u -m pytest -q --timeout 150 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" $O/pytest.err | head -30; tail -2 $O/pytest.err
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/r50_$i.log 2>$O/r50_$i.err; chk $? r50_$i; echo "r50_$i $(v r50_$i)"
done
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 8 > $O/vit.log 2>$O/vit.err; chk $? vit; echo "vit $(v vit)"
W="timeout -k 10 400 python scripts/bench_workloads.py --steps 40 --warmup 8"
for g in "" "--graph"; do
t=${g:+g}
$W --workload dcgan --mode native $g > $O/dcgan$t.log 2>$O/dcgan$t.err; chk $? dcgan$t; echo "dcgan$t $(v dcgan$t)"
$W --workload online --batch 8 --size 256 --mode native32 $g > $O/online32$t.log 2>$O/online32$t.err; chk $? online32$t; echo "online32$t $(v online32$t)"
$W --workload adain --batch 32 --size 256 --mode native $g > $O/adain$t.log 2>$O/adain$t.err; chk $? adain$t; echo "adain$t $(v adain$t)"
$W --workload nst --batch 1 --size 512 --mode native32 $g > $O/nst32$t.log 2>$O/nst32$t.err; chk $? nst32$t; echo "nst32$t $(v nst32$t)"
done
echo final rc=0
