# ViT-B/16 kernel summary after the norm-slot change (copies gone?)
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_43
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/p_vit -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 4 > $R/$O/p_vit.log 2>&1
chk $? p_vit
python3 $R/scripts/dbstats.py $R/$O/p_vit/run_results.db --steps 3 --top 40 --width 110 > $R/$O/vit_kernels.txt 2>&1; rm -f $R/$O/p_vit/run_results.db
head -30 $R/$O/vit_kernels.txt
