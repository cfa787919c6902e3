#!/bin/bash
# big-tile weight gradient per-shape timing under other partial caps / workgroup targets
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_28; mkdir -p $O; cd $R
TBAMD_WGRAD_CAP_MB=128 timeout -k 10 300 python -u scripts/tools/wgrad_big_ab.py > $O/cap128_wgs512.txt 2>&1 || exit $?
TBAMD_WGRAD_CAP_MB=128 TBAMD_WGRAD_BIG_WGS=256 timeout -k 10 300 python -u scripts/tools/wgrad_big_ab.py > $O/cap128_wgs256.txt 2>&1 || exit $?
TBAMD_WGRAD_CAP_MB=256 TBAMD_WGRAD_BIG_WGS=1024 timeout -k 10 300 python -u scripts/tools/wgrad_big_ab.py > $O/cap256_wgs1024.txt 2>&1 || exit $?
for f in cap128_wgs512 cap128_wgs256 cap256_wgs1024; do echo "== $f"; grep -v amdgpu.ids $O/$f.txt; done
