R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r22
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_linear.py tests/test_graph_step.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ln.log 2>&1
chk $? pytest_ln; tail -3 $O/pytest_ln.log
[ "$(grep -c failed $O/pytest_ln.log)" = "0" ] || exit 1
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 3 > $O/vit.log 2>$O/vit.err
chk $? vit; tail -1 $O/vit.log | cut -c1-300; grep "linear" $O/vit.err | head -20
TBAMD_GEMM_TABLE=none timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 3 > $O/vit_notable.log 2>$O/vit_notable.err
chk $? vit_notable; tail -1 $O/vit_notable.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 6 --warmup 3 > $R/$O/prof_vit.log 2>&1
chk $? prof
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err
chk $? bench; tail -1 $O/bench.log | cut -c1-200
