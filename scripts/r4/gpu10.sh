#!/bin/bash
# workloads with the route log (remaining vendor picks), ViT on the library-free GEMMs + trace,
# ResNet-50 kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_10; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --mode native --steps 30 --warmup 5 > $O/online.log 2>$O/online.err; chk $? online; tail -1 $O/online.log | cut -c1-140
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload online --batch 8 --size 256 --mode native32 --steps 30 --warmup 5 > $O/online32.log 2>$O/online32.err; chk $? online32; tail -1 $O/online32.log | cut -c1-140
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload adain --batch 32 --size 256 --mode native --steps 30 --warmup 5 > $O/adain.log 2>$O/adain.err; chk $? adain; tail -1 $O/adain.log | cut -c1-140
TBAMD_TUNE_LOG=1 timeout -k 10 500 python scripts/bench_workloads.py --workload nst --batch 1 --size 512 --mode native --steps 30 --warmup 5 > $O/nst.log 2>$O/nst.err; chk $? nst; tail -1 $O/nst.log | cut -c1-140
grep -h "\-> miopen" $O/*.err | sort | uniq > $O/miopen_routes.txt; echo "miopen routes: $(wc -l < $O/miopen_routes.txt)"; cut -c1-200 $O/miopen_routes.txt
timeout -k 10 400 python bench.py --model vit_b_16 --batch 128 --steps 20 --warmup 5 > $O/vit.log 2>$O/vit.err; chk $? vit; tail -1 $O/vit.log | cut -c1-150
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_vit -o vit -- python3 $R/bench.py --model vit_b_16 --batch 128 --steps 3 --warmup 3 > $O/tr_vit.err 2>&1; chk $? tr_vit
python3 $R/scripts/r4/qsplit.py $(find $O/tr_vit -name '*kernel_trace.csv') --top 30 > $O/vit_qsplit.txt; head -36 $O/vit_qsplit.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_r50 -o r50 -- python3 $R/bench.py --steps 4 --warmup 3 > $O/tr_r50.err 2>&1; chk $? tr_r50
python3 $R/scripts/r4/qsplit.py $(find $O/tr_r50 -name '*kernel_trace.csv') --top 40 > $O/r50_qsplit.txt; head -60 $O/r50_qsplit.txt
