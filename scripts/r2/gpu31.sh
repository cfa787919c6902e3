# VGG conv+ReLU epilogue fusion: tests; AdaIN / online / offline NST (bf16 graph + fp32) benches; DCGAN routes
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_31
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 300 python -u -m pytest tests/test_conv_relu_fusion.py tests/test_gpu_conv_any.py tests/test_gpu_aux_ops.py tests/test_gpu_examples.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -1 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest.log | head -60; kill $HB; exit 1; }
timeout -k 10 300 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 10 --warmup 3 --mode native > $O/adain_native.json 2> $O/adain_native.err
chk $? adain_native; cut -c1-200 $O/adain_native.json
timeout -k 10 300 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --steps 10 --warmup 3 --mode native > $O/online_native.json 2> $O/online_native.err
chk $? online_native; cut -c1-200 $O/online_native.json
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --size 512 --steps 20 --warmup 3 --mode native --graph > $O/nst_graph.json 2> $O/nst_graph.err
chk $? nst_graph; cut -c1-200 $O/nst_graph.json
timeout -k 10 300 python scripts/bench_workloads.py --workload nst --size 512 --steps 20 --warmup 3 --mode native32 > $O/nst_native32.json 2> $O/nst_native32.err
chk $? nst_native32; cut -c1-200 $O/nst_native32.json
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode native > $O/dcgan.json 2> $O/dcgan.err
chk $? dcgan; cut -c1-200 $O/dcgan.json; grep "conv-tune" $O/dcgan.err | grep -v "> native" | cut -c1-250
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --steps 20 --warmup 3 --mode native --graph > $O/dcgan_graph.json 2> $O/dcgan_graph.err
chk $? dcgan_graph; cut -c1-200 $O/dcgan_graph.json
kill $HB
