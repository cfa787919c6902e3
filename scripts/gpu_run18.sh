R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r18
O=gpurun_out/r18
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -v --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1
echo "attn pytest rc=$?"; tail -3 $O/pytest_attn.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>$O/bench.err || exit 1
echo "bench ok"; grep warmup $O/bench.err | head -2; tail -1 $O/bench.log
for m in native stock; do
  timeout -k 10 300 python scripts/bench_workloads.py --workload vit --mode $m --batch 128 --steps 10 --warmup 3 > $O/vit_$m.log 2>$O/vit_$m.err || exit 1
  tail -1 $O/vit_$m.log
  timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode $m --batch 128 --steps 20 --warmup 3 > $O/dcgan_$m.log 2>$O/dcgan_$m.err || exit 1
  tail -1 $O/dcgan_$m.log
done
for m in native stock stock32; do
  timeout -k 10 300 python scripts/bench_workloads.py --workload nst --mode $m --steps 20 --warmup 3 > $O/nst_$m.log 2>$O/nst_$m.err || exit 1
  tail -1 $O/nst_$m.log
done
