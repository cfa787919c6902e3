# device input pipeline: kernel vs reference tests, loaders, E2 ResNet-18 CIFAR b2048 end to end
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_11
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_data.py tests/test_gpu_examples.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest.log | head -80; exit 1; }
for L in none device; do
timeout -k 10 300 python scripts/bench_workloads.py --workload cifar --batch 2048 --steps 20 --warmup 5 --loader $L > $O/cifar_$L.json 2> $O/cifar_$L.err
chk $? cifar_$L; cat $O/cifar_$L.json
done
timeout -k 10 300 python scripts/bench_workloads.py --workload cifar --batch 2048 --steps 20 --warmup 5 --mode stock > $O/cifar_stock.json 2> $O/cifar_stock.err
chk $? cifar_stock; cat $O/cifar_stock.json
