# full GPU suite; DCGAN (generic edge convs, graph), ViT (fast GELU), ResNet-50
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_16
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest_gpu; tail -2 $O/pytest_gpu.log
[ "$(grep -c FAILED $O/pytest_gpu.log)" = "0" ] || { grep -m3 -B5 -A30 "Error\|assert" $O/pytest_gpu.log | head -60; }
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cut -c1-200 $O/bench.json
for M in native stock; do
TBAMD_TUNE_LOG=1 timeout -k 10 240 python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 20 --warmup 3 --mode $M > $O/dcgan_$M.json 2> $O/dcgan_$M.err
chk $? dcgan_$M; cut -c1-200 $O/dcgan_$M.json
done
timeout -k 10 240 python scripts/bench_workloads.py --workload dcgan --batch 128 --steps 20 --warmup 3 --graph > $O/dcgan_graph.json 2> $O/dcgan_graph.err
echo dcgan_graph rc=$?; cut -c1-200 $O/dcgan_graph.json; tail -3 $O/dcgan_graph.err
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cut -c1-200 $O/vit.json
