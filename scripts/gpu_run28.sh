R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r28
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_layernorm.py tests/test_gpu_linear.py tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -2 $O/pytest.log
[ "$(grep -c failed $O/pytest.log)" = "0" ] || exit 1
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 3 > $O/vit.log 2>$O/vit.err
chk $? vit; tail -1 $O/vit.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 6 --warmup 3 > $R/$O/prof_vit.log 2>&1
chk $? prof
