# LN backward with dadd prefetched: LN numerics, ViT bench x2, ViT kernel summary
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_44
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 0) ;; *) tail -30 $O/$2.err 2>/dev/null; exit $rc;; esac; }
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_layernorm.py tests/test_gpu_kernels.py > $O/pytest.err 2>&1
chk $? pytest; tail -1 $O/pytest.err
for i in 1 2; do
timeout -k 10 300 python -u bench.py --model vit_b_16 --batch 128 --steps 12 --warmup 4 > $O/vit_$i.json 2>$O/vit_$i.err
chk $? vit_$i; cut -c1-160 $O/vit_$i.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 4 > $R/$O/p_vit.log 2>&1
chk $? p_vit
python3 $R/scripts/dbstats.py $R/$O/p_vit/run_results.db --steps 3 --top 40 --width 110 > $R/$O/vit_kernels.txt 2>&1; rm -f $R/$O/p_vit/run_results.db
grep -E "steps=|ln_bwd|ln_fwd" $R/$O/vit_kernels.txt
