# native GELU forward (ViT fc1), DCGAN edge dgrads: tests; ViT bench + kernel summary
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_35
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest tests/test_gpu_aux_ops.py tests/test_gpu_conv_any.py tests/test_gpu_linear.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cut -c1-200 $O/vit.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 4 > $R/$O/p_vit.log 2>&1
chk $? p_vit
python3 $R/scripts/dbstats.py $R/$O/p_vit/run_results.db --steps 3 --top 40 --width 110 > $R/$O/vit_kernels.txt 2>&1; rm -f $R/$O/p_vit/run_results.db
kill $HB
