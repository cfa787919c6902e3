# round 2, run 4 (re-entry): full GPU suite, ResNet-50 bench, ViT-B/16 bench + kernel stats, GEMM engine vs hipBLASLt
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_04
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest_gpu; tail -3 $O/pytest_gpu.log
[ "$(grep -c FAILED $O/pytest_gpu.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest_gpu.log | head -80; }
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
chk $? bench; cut -c1-200 $O/bench.json
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cut -c1-220 $O/vit.json; grep gemm-tune $O/vit.err | head -20
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vit -o vit -- python bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/prof_vit.log 2>&1
chk $? prof_vit
python scripts/steady.py $O/prof_vit/vit_kernel_trace.csv 3 > $O/vit_steady.txt; head -30 $O/vit_steady.txt
timeout -k 10 300 python -u scripts/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err
chk $? gemm_bench
python - <<'PY'
import json
for l in open("gpurun_out/r2_04/gemm_bench.jsonl"):
    d=json.loads(l)
    kind = "wgrad" if d.get("wgrad") else f"tw={int(d['tw'])}"
    print(f"{d['shape']:15s} {kind:5s} best t{d['best_tile']} {d['ms']:.4f}ms {d['tflops']:7.1f}TF torch {d['torch_ms']:.4f} {d['torch_tflops']:7.1f}TF")
PY
