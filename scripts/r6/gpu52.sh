#!/bin/bash
# BN apply cap 2048 (old) vs 16384 (new default): DCGAN-128 and ResNet-101, alternated 3x
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_52; mkdir -p $O; cd $R
b() { n=$1; shift; timeout -k 10 300 "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; }
for i in 1 2 3; do
for wg in 2048 16384; do
TBAMD_BN_APPLY_WG=$wg b dcgan python scripts/bench_workloads.py --workload dcgan --steps 60 --warmup 10
TBAMD_BN_APPLY_WG=$wg b r101 python bench.py --model resnet101 --steps 20
echo "wg=$wg dcgan $(tail -1 $O/dcgan.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'])") r101 $(python3 -c "import json;d=json.load(open('$O/r101.json'));print(d['value'])")"
done
done
