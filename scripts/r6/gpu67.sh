#!/bin/bash
# closing tree over long timed windows: 100 and 300 steps (memory stays flat, throughput holds)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6_67; mkdir -p $O; cd $R
for s in 20 100 300; do
timeout -k 10 400 python bench.py --steps $s --warmup 5 > $O/b_$s.json 2> $O/b_$s.err || exit $?
echo "steps=$s $(python3 -c "import json;d=json.load(open('$O/b_$s.json'));print(d['value'],d['ms_per_step'],d['final_loss'])")"
done
