#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_11; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/tools/mem_probe.py > $O/mem.txt 2> $O/mem.err; rc=$?; cat $O/mem.txt; tail -3 $O/mem.err; [ $rc -eq 0 ] || exit $rc
b() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.json 2> $O/$n.err || exit $?; echo "$n $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['ms_per_step'])")"; }
b colsum_new_1 --steps 20 --warmup 5
b colsum_new_2 --steps 20 --warmup 5
