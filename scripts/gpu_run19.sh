R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r19
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_attention.py -x -v --timeout 120 --timeout-method thread > $O/pytest_gram.log 2>&1
echo "gram pytest rc=$?"; tail -3 $O/pytest_gram.log
timeout -k 10 300 python scripts/bench_workloads.py --workload vit --mode stock --batch 128 --steps 10 --warmup 3 > $O/vit_stock.log 2>$O/vit_stock.err || exit 1
tail -1 $O/vit_stock.log
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode stock --batch 128 --steps 20 --warmup 3 > $O/dcgan_stock.log 2>$O/dcgan_stock.err || exit 1
tail -1 $O/dcgan_stock.log
for m in native stock stock32; do
  timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode $m --steps 20 --warmup 3 > $O/nst_$m.log 2>$O/nst_$m.err || exit 1
  tail -1 $O/nst_$m.log
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 6 --warmup 3 > $R/$O/prof_vit.log 2>&1
echo "prof rc=$?"
