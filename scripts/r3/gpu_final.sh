#!/bin/bash
# round-3 closing check on the committed tree: full GPU suite, smoke, headline bench as the driver
# runs it, ViT-B/16, and a whole-step kernel trace of the headline
set -o pipefail
O=gpurun_out/r3_final; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.err 2>&1 ; chk $? pytest; tail -2 $O/pytest.err
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.err 2>&1; chk $? smoke; tail -1 $O/smoke.err
timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 10 > $O/r50.log 2>$O/r50.err; chk $? r50; tail -1 $O/r50.log | cut -c1-200
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r50 -- python bench.py --steps 4 --warmup 3 > $O/prof.log 2>&1
chk $? prof
