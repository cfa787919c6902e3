#!/bin/bash
# round-4 opening measurement on the round-3 tree: headline bench, ViT bench, whole-step kernel
# traces (ResNet-50, ViT-B/16) and three PMC passes of the ResNet-50 step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_01; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python bench.py --gpus 1 --steps 30 --warmup 10 > $O/r50.log 2>$O/r50.err; chk $? r50; tail -1 $O/r50.log | cut -c1-200
timeout -k 10 300 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_r50 -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr_r50.err 2>&1; chk $? tr_r50
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_vit -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 4 --warmup 3 > $O/tr_vit.err 2>&1; chk $? tr_vit
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_sq.err 2>&1; chk $? pmc_sq
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_fetch.err 2>&1; chk $? pmc_fetch
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_write.err 2>&1; chk $? pmc_write
for p in pmc_sq pmc_fetch pmc_write; do
  [ -f $O/$p/run_counter_collection.csv ] || { f=$(find $O/$p -name '*counter_collection.csv' | head -1); [ -n "$f" ] && mv "$f" $O/$p/run_counter_collection.csv; }
done
python3 $R/scripts/pmc_summary.py $O 453 > $O/r50_pmc_summary.txt 2>&1
head -40 $O/r50_pmc_summary.txt | cut -c1-130
# keep the kernel-trace CSVs (small); drop the PMC ones
find $O/pmc_* -name '*.csv' -delete; find $O -name '*.db' -delete
du -sh $O
