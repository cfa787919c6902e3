#!/bin/bash
# dgrad-epilogue k-loop pipelining A/B (TBAMD_CONV_EPI_STAGES 1 / 2 / 3): per-shape + whole step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_06; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -40 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
for s in 1 2 3; do
TBAMD_CONV_EPI_STAGES=$s timeout -k 10 300 python scripts/r4/conv1x1_bench.py > $O/c_s$s.log 2>$O/c_s$s.err; chk $? c_s$s
done
paste -d' ' <(cut -c1-90 $O/c_s1.log) <(cut -c40-90 $O/c_s2.log) <(cut -c40-90 $O/c_s3.log) | grep dgrad
for i in 1 2; do
for s in 1 2 3; do
TBAMD_CONV_EPI_STAGES=$s timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/b_s$s.$i.log 2>$O/b_s$s.$i.err; chk $? b_s$s.$i; echo "stages $s: $(tail -1 $O/b_s$s.$i.log | cut -c1-120)"
done
done
for s in 2 3; do
TBAMD_CONV_STAGES=$s timeout -k 10 300 python scripts/r4/conv1x1_bench.py > $O/f_s$s.log 2>$O/f_s$s.err; chk $? f_s$s
done
paste -d' ' <(cut -c1-90 $O/c_s1.log) <(cut -c40-90 $O/f_s2.log) <(cut -c40-90 $O/f_s3.log) | grep -v dgrad
for s in 2 3; do
TBAMD_CONV_STAGES=$s timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bf_s$s.log 2>$O/bf_s$s.err; chk $? bf_s$s; echo "fwd stages $s: $(tail -1 $O/bf_s$s.log | cut -c1-120)"
done
for wv in 1 0.5 0.25; do
TBAMD_WGRAD_WAVES=$wv timeout -k 10 300 python scripts/r4/wgrad_bench.py > $O/wg_$wv.log 2>$O/wg_$wv.err; chk $? wg_$wv
done
paste -d' ' <(cut -c1-100 $O/wg_1.log) <(cut -c50-100 $O/wg_0.5.log) <(cut -c50-100 $O/wg_0.25.log)
for wv in 0.5 0.25; do
TBAMD_WGRAD_WAVES=$wv timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/bw_$wv.log 2>$O/bw_$wv.err; chk $? bw_$wv; echo "wgrad waves $wv: $(tail -1 $O/bw_$wv.log | cut -c1-120)"
done
