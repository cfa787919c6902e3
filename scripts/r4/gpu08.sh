#!/bin/bash
# closing-style workload A/B (DCGAN native vs stock, alternated) with the route log (remaining
# MIOpen picks), online / AdaIN NST native runs, and three PMC passes of the ResNet-50 step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_08; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
TBAMD_TUNE_LOG=1 timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode native --steps 60 --warmup 10 > $O/dnat$i.log 2>$O/dnat$i.err; chk $? dnat$i; tail -1 $O/dnat$i.log | cut -c1-140
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode stock --steps 60 --warmup 10 > $O/dstock$i.log 2>$O/dstock$i.err; chk $? dstock$i; tail -1 $O/dstock$i.log | cut -c1-140
done
for w in online adain; do
TBAMD_TUNE_LOG=1 timeout -k 10 400 python scripts/bench_workloads.py --workload $w --mode native --steps 20 --warmup 5 > $O/$w.log 2>$O/$w.err; chk $? $w; tail -1 $O/$w.log | cut -c1-140
done
grep -h "\-> miopen" $O/*.err | sort | uniq > $O/miopen_routes.txt; echo "miopen routes: $(wc -l < $O/miopen_routes.txt)"; cat $O/miopen_routes.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_sq.err 2>&1; chk $? pmc_sq
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_fetch.err 2>&1; chk $? pmc_fetch
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 3 > $O/pmc_write.err 2>&1; chk $? pmc_write
for p in pmc_sq pmc_fetch pmc_write; do
  [ -f $O/$p/run_counter_collection.csv ] || { f=$(find $O/$p -name '*counter_collection.csv' | head -1); [ -n "$f" ] && mv "$f" $O/$p/run_counter_collection.csv; }
done
N=$(python3 $R/scripts/r4/step_dispatches.py $O/pmc_sq/run_counter_collection.csv)
python3 $R/scripts/pmc_summary.py $O $N > $O/r50_pmc_summary.txt 2>&1
head -45 $O/r50_pmc_summary.txt | cut -c1-130
find $O/pmc_* -name '*.csv' -delete; find $O -name '*.db' -delete
cd $R
# the ResNet example on its ImageNet config (1 GPU, b256) vs bench.py: throughput within 2 %
cat > $O/r50ex.yml <<YML
#include $R/examples/img_cls/resnet/resnet50_imagenet.yml
env:
  fp16: true
  n_gpu: 1
  distributed: false
dataset:
  name: imagenet
  root: /nonexistent/imagenet
loader:
  batch_size: 256
  num_workers: 0
  pin_memory: false
  drop_last: true
YML
TBAMD_CONFIG=$O/r50ex.yml TBAMD_EXAMPLE_MAX_ITERS=50 TBAMD_EXAMPLE_TIMING=20 timeout -k 10 500 python examples/img_cls/resnet/resnet.py > $O/r50ex.log 2>$O/r50ex.err; chk $? r50ex; grep example_img_s $O/r50ex.log
timeout -k 10 300 python bench.py --steps 30 --warmup 20 > $O/r50b.log 2>$O/r50b.err; chk $? r50b; tail -1 $O/r50b.log | cut -c1-150
