#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_12; mkdir -p $O; cd $R
timeout -k 10 300 python -u scripts/tools/leak_probe.py > $O/leak.txt 2> $O/leak.err; rc=$?; cat $O/leak.txt; tail -3 $O/leak.err; exit $rc
