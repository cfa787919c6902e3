#!/bin/bash
# whole-step hipGraph replay (GraphedStep) vs eager on the current tree, with and without the
# weight-gradient side stream inside the capture
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_08; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/eager_$i.log 2>$O/eager_$i.err; chk $? eager_$i; echo "eager_$i $(v eager_$i)"
timeout -k 10 300 python bench.py --graph on > $O/graph_$i.log 2>$O/graph_$i.err; chk $? graph_$i; echo "graph_$i $(v graph_$i)"
TBAMD_WGRAD_STREAM_CAPTURE=1 timeout -k 10 300 python bench.py --graph on > $O/graphs_$i.log 2>$O/graphs_$i.err; chk $? graphs_$i; echo "graphs_$i $(v graphs_$i)"
done
echo final rc=0
