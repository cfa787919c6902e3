# conv forward tile-shape study (128x128 vs 128x256 vs 256x128) + PMC of a 3x3 and a 1x1 shape
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_25
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
timeout -k 10 300 python -u scripts/r2/conv_bk_tune.py > $O/tune.jsonl 2> $O/tune.err
chk $? tune; tail -1 $O/tune.jsonl | cut -c1-400
cd /tmp && export TMPDIR=/tmp
for v in "128 28 128 3 1 0 0 0 20 0" "128 28 128 3 1 0 0 0 20 1" "1024 14 256 1 1 0 0 0 20 0" "1024 14 256 1 1 0 0 0 20 2"; do
  tag=$(echo $v | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/$O/pmc_$tag -o run -- python3 $R/scripts/r2/conv_one.py $v > $R/$O/pmc_$tag.log 2>&1
  chk $? pmc_$tag
done
