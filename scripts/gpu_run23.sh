R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r23
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_layernorm.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ln.log 2>&1
chk $? pytest_ln; tail -2 $O/pytest_ln.log
[ "$(grep -c failed $O/pytest_ln.log)" = "0" ] || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 6 --warmup 3 > $R/$O/prof_vit.log 2>&1
chk $? prof; cd $R; tail -1 $O/prof_vit.log | cut -c1-200
for w in dcgan nst; do
  timeout -k 10 300 python scripts/bench_workloads.py --workload $w --mode native --steps 20 --warmup 4 > $O/${w}_native.log 2>$O/${w}_native.err
  chk $? ${w}_native; tail -1 $O/${w}_native.log | cut -c1-200
  timeout -k 10 300 python scripts/bench_workloads.py --workload $w --mode native --graph --steps 20 --warmup 4 > $O/${w}_graph.log 2>$O/${w}_graph.err
  chk $? ${w}_graph; tail -1 $O/${w}_graph.log | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_dcgan -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --mode native --steps 10 --warmup 3 > $R/$O/prof_dcgan.log 2>&1
chk $? prof_dcgan
