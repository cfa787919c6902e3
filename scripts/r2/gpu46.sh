# ResNet-50 whole-step PMC (MFMA busy, LDS conflicts, HBM bytes per kernel) on the round-2 closing tree
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2_46
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 0) ;; *) tail -5 $O/$2.log; exit $rc;; esac; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_sq.log 2>&1
chk $? pmc_sq
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_fetch.log 2>&1
chk $? pmc_fetch
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_write.log 2>&1
chk $? pmc_write
for p in pmc_sq pmc_fetch pmc_write; do
  [ -f $O/$p/run_counter_collection.csv ] || { f=$(find $O/$p -name '*counter_collection.csv' | head -1); [ -n "$f" ] && mv "$f" $O/$p/run_counter_collection.csv; }
done
python3 $R/scripts/pmc_summary.py $O 453 > $O/r50_pmc_summary.txt 2>&1
cat $O/r50_pmc_summary.txt | cut -c1-130
find $O -name '*.csv' -delete; find $O -name '*.db' -delete
du -sh $O
