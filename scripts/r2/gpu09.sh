# full GPU suite + ViT bench (native/hipBLASLt per-shape GEMM routing) + ResNet bench
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_09
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
TBAMD_TUNE_LOG=1 timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 10 --warmup 4 > $O/vit.json 2> $O/vit.err
chk $? vit; cut -c1-220 $O/vit.json; grep gemm-tune $O/vit.err | head -20
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
chk $? pytest_gpu; tail -3 $O/pytest_gpu.log
[ "$(grep -c FAILED $O/pytest_gpu.log)" = "0" ] || { grep -m5 -B5 -A40 "Error\|assert" $O/pytest_gpu.log | head -80; }
