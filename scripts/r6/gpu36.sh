#!/bin/bash
# streaming bandwidth probe: 2-read / 1-write bf16 stream, load/store forms and grid shapes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_36; mkdir -p $O; cd $R
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/membw_probe scripts/tools/membw_probe.hip || exit $?
timeout -k 10 120 /tmp/membw_probe > $O/membw.txt 2>&1; rc=$?; cat $O/membw.txt; exit $rc
