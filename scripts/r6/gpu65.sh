#!/bin/bash
# native vs stock on ONE box for the style-transfer / CIFAR workloads (BASELINE config 4 and E2/E5-E7);
# heartbeat for MIOpen's first-use compiles
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_65; mkdir -p $O; cd $R
( while sleep 30; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
val() { tail -1 $1 | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d.get("value", d.get("img_s")))'; }
W="python scripts/bench_workloads.py --steps 30 --warmup 6"
run() { n=$1; shift; timeout -k 10 900 $W "$@" > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }; }
run nst_n32 --workload nst --batch 1 --size 512 --mode native32
run nst_s32 --workload nst --batch 1 --size 512 --mode stock32
echo "nst fp32 native $(val $O/nst_n32.json) stock $(val $O/nst_s32.json)"
run adain_n --workload adain --batch 32 --size 256 --mode native
run adain_s --workload adain --batch 32 --size 256 --mode stock
echo "adain bf16 native $(val $O/adain_n.json) stock $(val $O/adain_s.json)"
run online_n --workload online --batch 8 --size 256 --mode native
run online_s --workload online --batch 8 --size 256 --mode stock
echo "online bf16 native $(val $O/online_n.json) stock $(val $O/online_s.json)"
run cifar_n --workload cifar --loader device --batch 2048 --mode native
run cifar_s --workload cifar --loader device --batch 2048 --mode stock
echo "cifar native $(val $O/cifar_n.json) stock $(val $O/cifar_s.json)"
