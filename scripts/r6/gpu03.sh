#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_03; mkdir -p $O; cd $R
timeout -k 10 300 python scripts/tools/vit_gemm_tail.py > $O/tail.jsonl 2> $O/tail.err; rc=$?; cat $O/tail.jsonl; exit $rc
