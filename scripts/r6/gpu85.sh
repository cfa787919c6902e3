#!/bin/bash
# DDP wrapper serialisation: under RCCL the side stream lands on the compute stream's hardware queue (r6_84 trace).
# --ddp with the default side stream / TBAMD_SIDE_PRIORITY=low (its own queue class) / GPU_MAX_HW_QUEUES=8; plain for scale
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_85; mkdir -p $O; cd $R
run() { n=$1; shift; E=(); ARGS=(); for x in "$@"; do case $x in --*) ARGS+=("$x");; *) E+=("$x");; esac; done
env "${E[@]}" timeout -k 10 300 python bench.py --steps 20 --warmup 5 "${ARGS[@]}" > $O/$n.out 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
echo "$n $(grep '^{' $O/$n.out | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'])")"; }
for i in 1 2; do
run plain A=1
run ddp_default A=1 --ddp
run ddp_low TBAMD_SIDE_PRIORITY=low --ddp
run ddp_q8 GPU_MAX_HW_QUEUES=8 --ddp
run plain_q8 GPU_MAX_HW_QUEUES=8
done
