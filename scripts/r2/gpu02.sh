# round 2, run 2: native GEMM engine numerics + timing vs hipBLASLt
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_02
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 240 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > $O/pytest_gemm.log 2>&1
chk $? pytest_gemm; tail -3 $O/pytest_gemm.log
[ "$(grep -c FAILED $O/pytest_gemm.log)" = "0" ] || { grep -m3 -A30 "Error\|assert" $O/pytest_gemm.log | head -60; exit 1; }
timeout -k 10 300 python -u scripts/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err
chk $? gemm_bench
python - <<'PY'
import json
for l in open("gpurun_out/r2_02/gemm_bench.jsonl"):
    d=json.loads(l)
    kind = "wgrad" if d.get("wgrad") else f"tw={int(d['tw'])}"
    print(f"{d['shape']:15s} {kind:5s} best t{d['best_tile']} {d['ms']:.4f}ms {d['tflops']:7.1f}TF  torch {d['torch_ms']:.4f}ms {d['torch_tflops']:7.1f}TF  {d['all_ms']}")
PY
