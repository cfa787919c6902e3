# round 2, run 5: ping-pong GEMM correctness + timing; nativize fix
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_${RUN:-05}
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u scripts/r2/pp_bench.py > $O/pp.jsonl 2> $O/pp.err
chk $? pp_bench; tail -5 $O/pp.err
python scripts/r2/pp_sum.py $O/pp.jsonl
timeout -k 10 240 python -u -m pytest tests/test_gpu_nativize.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cut -c1-200 $O/bench.json
