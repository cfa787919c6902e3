# round 2, run 3: Linear on the native GEMM engine -> linear/examples tests, ViT-B/16 bench + kernel stats
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_03
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_r2_correctness.py tests/test_gpu_nativize.py tests/test_gpu_gemm.py tests/test_gpu_linear.py tests/test_gpu_examples.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
chk $? pytest; tail -3 $O/pytest.log
[ "$(grep -c FAILED $O/pytest.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest.log | head -80; exit 1; }
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cat $O/vit.json | cut -c1-220; grep gemm-tune $O/vit.err | head -20
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vit -o vit -- python bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/prof_vit.log 2>&1
chk $? prof_vit
python scripts/steady.py $O/prof_vit/vit_kernel_trace.csv 3 > $O/vit_steady.txt; head -40 $O/vit_steady.txt
timeout -k 10 300 python -u scripts/gemm_bench.py > $O/gemm_bench.jsonl 2> $O/gemm_bench.err
chk $? gemm_bench
python - <<'PY'
import json
for l in open("gpurun_out/r2_03/gemm_bench.jsonl"):
    d=json.loads(l)
    kind = "wgrad" if d.get("wgrad") else f"tw={int(d['tw'])}"
    a = d['all_ms']; old = min(v for k, v in a.items() if int(k) < 10); new = min(v for k, v in a.items() if int(k) >= 10)
    print(f"{d['shape']:15s} {kind:5s} best t{d['best_tile']} {d['ms']:.4f}ms {d['tflops']:7.1f}TF torch {d['torch_ms']:.4f} {d['torch_tflops']:7.1f}TF  old {old:.4f} split-half {new:.4f}")
PY
