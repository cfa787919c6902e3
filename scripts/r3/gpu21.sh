#!/bin/bash
# secondary workloads native vs stock at the reference precision (fp32 NST) and DCGAN bf16;
# kernel trace of the fp32 online style-transfer step
set -o pipefail
O=gpurun_out/r3_21; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
for w in online adain nst; do for m in native32 stock32; do
TBAMD_TUNE_LOG=1 timeout -k 10 600 python scripts/bench_workloads.py --workload $w --mode $m --save-routes $O/routes_${w}_$m.json > $O/${w}_$m.log 2>$O/${w}_$m.err; chk $? ${w}_$m; tail -1 $O/${w}_$m.log | cut -c1-160
done; done
for m in native stock; do
timeout -k 10 300 python scripts/bench_workloads.py --workload dcgan --mode $m > $O/dcgan_$m.log 2>$O/dcgan_$m.err; chk $? dcgan_$m; tail -1 $O/dcgan_$m.log | cut -c1-160
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o online32 -- python scripts/bench_workloads.py --workload online --mode native32 --steps 6 --warmup 4 > $O/prof.log 2>&1
chk $? prof
