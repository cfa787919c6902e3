# Fresh-container re-check: full GPU suite, smoke, 1-GPU bench, kernel stats of the bench step
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_23
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
timeout -k 10 120 python __graft_entry__.py > $O/smoke.log 2>&1
chk $? smoke; tail -1 $O/smoke.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cut -c1-300 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 5 > $R/$O/prof.log 2>&1
chk $? prof
kill $HB
