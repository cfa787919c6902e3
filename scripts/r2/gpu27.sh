# kernel profiles of the AdaIN (E7) native/stock steps and the DCGAN native step
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_27
mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; case $rc in 124|134|137|139) kill $HB 2>/dev/null; exit $rc;; esac; }
( while true; do sleep 50; date >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 200 python -u -m pytest tests/test_gpu_aux_ops.py -x -q --timeout 120 --timeout-method thread > $O/pytest_aux.log 2>&1
chk $? pytest_aux; tail -1 $O/pytest_aux.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/adain_native -o run -- python3 $R/scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 4 --warmup 3 --mode native > $R/$O/adain_native.json 2> $R/$O/adain_native.err
chk $? adain_native; cut -c1-200 $R/$O/adain_native.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/adain_stock -o run -- python3 $R/scripts/bench_workloads.py --workload adain --batch 32 --size 256 --steps 4 --warmup 3 --mode stock > $R/$O/adain_stock.json 2> $R/$O/adain_stock.err
chk $? adain_stock; cut -c1-200 $R/$O/adain_stock.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/dcgan -o run -- python3 $R/scripts/bench_workloads.py --workload dcgan --steps 4 --warmup 3 --mode native > $R/$O/dcgan.json 2> $R/$O/dcgan.err
chk $? dcgan; cut -c1-200 $R/$O/dcgan.json
kill $HB
