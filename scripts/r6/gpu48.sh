#!/bin/bash
# BN apply grid (old 2048 vs new full grid) on the deeper ResNets and CIFAR ResNet-18, alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_48; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; }
for i in 1 2; do
for wg in 2048 131072; do
TBAMD_BN_APPLY_WG=$wg b r101 python bench.py --model resnet101 --steps 20
TBAMD_BN_APPLY_WG=$wg b r152 python bench.py --model resnet152 --steps 10
TBAMD_BN_APPLY_WG=$wg b cifar python scripts/bench_workloads.py --workload cifar --loader device --batch 2048 --steps 40 --warmup 8
echo "wg=$wg r101 $(python3 -c "import json;d=json.load(open('$O/r101.json'));print(d['value'])") r152 $(python3 -c "import json;d=json.load(open('$O/r152.json'));print(d['value'])") cifar $(tail -1 $O/cifar.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['img_s'])")"
done
done
