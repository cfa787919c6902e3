#!/bin/bash
# weight-gradient occupancy 2 (default) vs 3 on the full-grid BN tree: ResNet-50 x3 and DCGAN-128 x2, alternated
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_44; mkdir -p $O; cd $R
run() { env "$@" timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?; python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])"; }
rund() { env "$@" timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 40 --warmup 8 > $O/d.json 2> $O/d.err || exit $?; tail -1 $O/d.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])"; }
for i in 1 2 3; do
echo "r50 wocc2  $(run X=1)"
echo "r50 wocc3  $(run TBAMD_WGRAD_OCC=3)"
done
for i in 1 2; do
echo "dcgan wocc2  $(rund X=1)"
echo "dcgan wocc3  $(rund TBAMD_WGRAD_OCC=3)"
done
