#!/bin/bash
# XF restricted to bn2 -> persistent conv3 (TBAMD_BN_XF=2) A/B; closing whole-step PMC of the
# ResNet-50 step (3 passes) and of the ViT-B/16 step (3 passes) on the round-4 tree
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_15; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
b() { timeout -k 10 300 python bench.py --steps 30 --warmup 10 "${@:2}" > $O/$1.log 2>$O/$1.err; chk $? $1; echo "$1 $(tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
for i in 1 2; do
TBAMD_BN_XF=2 b xf2_$i
TBAMD_BN_XF=0 b off_$i
done
cd /tmp && export TMPDIR=/tmp
pmc() {  # name, dispatches/step, bench args...
  local n=$1 d=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/$n/pmc_sq -o run -- python3 $R/bench.py --steps 2 --warmup 3 "$@" > $O/${n}_sq.err 2>&1; chk $? ${n}_sq
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/$n/pmc_fetch -o run -- python3 $R/bench.py --steps 2 --warmup 3 "$@" > $O/${n}_fetch.err 2>&1; chk $? ${n}_fetch
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/$n/pmc_write -o run -- python3 $R/bench.py --steps 2 --warmup 3 "$@" > $O/${n}_write.err 2>&1; chk $? ${n}_write
  for p in pmc_sq pmc_fetch pmc_write; do
    [ -f $O/$n/$p/run_counter_collection.csv ] || { f=$(find $O/$n/$p -name '*counter_collection.csv' | head -1); [ -n "$f" ] && mv "$f" $O/$n/$p/run_counter_collection.csv; }
  done
  python3 $R/scripts/pmc_summary.py $O/$n $d > $O/${n}_pmc_summary.txt 2>&1
  head -30 $O/${n}_pmc_summary.txt | cut -c1-130
  find $O/$n -name '*.csv' -delete; find $O -name '*.db' -delete
}
pmc r50 453
pmc vit 422 --model vit_b_16 --batch 128
echo final rc=0
