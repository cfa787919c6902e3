#!/bin/bash
# occupancy knobs re-checked on the full-grid BN tree (step A/B alternated)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_43; mkdir -p $O; cd $R
run() { env "$@" timeout -k 10 300 python bench.py --steps 30 > $O/b.json 2> $O/b.err || exit $?; python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'],d['ms_per_step'])"; }
for i in 1 2; do
echo "default              $(run X=1)"
echo "conv occ 3           $(run TBAMD_CONV_OCC=3)"
echo "wgrad occ 3          $(run TBAMD_WGRAD_OCC=3)"
done
