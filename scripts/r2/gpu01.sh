# round 2, run 1: GPU suite + bench (plain / native DDP forced on a 1-rank RCCL group, bf16 and f32 reduce)
# + a kernel trace of the DDP step (RCCL kernels interleaved with backward)
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_01
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest_gpu; tail -3 $O/pytest_gpu.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cat $O/bench.json | cut -c1-200
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --ddp > $O/bench_ddp.json 2> $O/bench_ddp.err
chk $? bench_ddp; cat $O/bench_ddp.json | cut -c1-200; grep "ddp buckets" $O/bench_ddp.err
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --ddp --reduce-dtype fp32 > $O/bench_ddp32.json 2> $O/bench_ddp32.err
chk $? bench_ddp32; cat $O/bench_ddp32.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ddp -o ddp -- python bench.py --steps 4 --warmup 3 --ddp > $O/prof_ddp.log 2>&1
chk $? prof_ddp
find $O/prof_ddp -name "*.csv" | head
