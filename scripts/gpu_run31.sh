R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r31
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "stem or stride2" > $O/pytest_stem.log 2>&1
chk $? pytest_stem; tail -2 $O/pytest_stem.log
[ "$(grep -c failed $O/pytest_stem.log)" = "0" ] || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread --deselect tests/test_gpu_examples.py > $O/pytest_gpu.log 2>&1
chk $? pytest; tail -2 $O/pytest_gpu.log
[ "$(grep -c failed $O/pytest_gpu.log)" = "0" ] || exit 1
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err
chk $? bench; tail -1 $O/bench.log | cut -c1-220; grep stem $O/bench.err | head -3
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_rn50 -o run -- python3 $R/bench.py --steps 6 --warmup 4 > $R/$O/prof_rn50.log 2>&1
chk $? prof
