#!/bin/bash
# closing re-measure of the family / secondary workloads on the full-grid BN tree (native only)
# stock comparators are unchanged stacks, profiles/r04_family)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_47; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
b resnet50 --steps 20 --warmup 5
b stock_resnet50 --model stock_resnet50 --steps 20 --warmup 5
for m in resnet18 resnet34 resnet101 resnet152; do b $m --model $m --steps 20 --warmup 5; done
b vit_s_16 --model vit_s_16 --batch 128 --steps 20 --warmup 5
b vit_b_16 --model vit_b_16 --batch 128 --steps 20 --warmup 5
w() { n=$1; shift; timeout -k 10 300 python scripts/bench_workloads.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(tail -1 $O/$n.json | cut -c1-220)"; }
w dcgan --workload dcgan
w nst --workload nst --mode native32
w cifar --workload cifar --loader device --batch 2048
w adain --workload adain --batch 32 --size 256
w online --workload online --batch 8 --size 256
timeout -k 10 400 python scripts/tools/lmdb_e2e.py > $O/lmdb.json 2> $O/lmdb.err || exit $?; echo "lmdb $(cut -c1-240 $O/lmdb.json)"
