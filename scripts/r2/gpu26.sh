# conv forward scheduling (iglp_opt) study; BN colsum slicing sweep on the bench; ViT kernel profile
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_26
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u scripts/r2/conv_bk_tune.py > $O/tune.jsonl 2> $O/tune.err
chk $? tune; tail -1 $O/tune.jsonl | cut -c1-400
for cs in "64,64" "16,256" "32,128" "24,512"; do
  TBAMD_COLSUM=$cs timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench_cs_$cs.json 2> $O/bench_cs_$cs.err
  chk $? bench_cs_$cs; cut -c1-200 $O/bench_cs_$cs.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/vitprof -o run -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 4 > $R/$O/vitprof.log 2>&1
chk $? vitprof
