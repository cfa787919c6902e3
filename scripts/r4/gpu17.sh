#!/bin/bash
# A-fragment prefetch schedule for the smaller conv tiles (TBAMD_CONV_SCHED A/B), the example after
# the device-resident normalisation constants, DCGAN native/stock, and the touched GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4_17; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -eq 0 ] || exit $rc; }
chkt() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $O/$2.err | head -20; [ $rc -le 1 ] || exit $rc; }
v() { tail -1 $O/$1.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 700 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_convgemm.py tests/test_gpu_conv1x1p.py tests/test_gpu_xf.py tests/test_gpu_ddp.py tests/test_gpu_data.py tests/test_gpu_trajectory.py tests/test_gpu_example_resnet.py -s > $O/t.err 2>&1; chkt $? t; grep -E "passed|failed|deviation" $O/t.err | tail -6
for i in 1 2; do
TBAMD_CONV_SCHED=1 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/s1_$i.log 2>$O/s1_$i.err; chk $? s1_$i; echo "s1_$i $(v s1_$i)"
TBAMD_CONV_SCHED=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > $O/s0_$i.log 2>$O/s0_$i.err; chk $? s0_$i; echo "s0_$i $(v s0_$i)"
done
cat > $O/r50ex.yml <<YML
#include $R/examples/img_cls/resnet/resnet50_imagenet.yml
env:
  fp16: true
  n_gpu: 1
  distributed: false
dataset:
  name: synthetic:imagenet
  root: /nonexistent/imagenet
loader:
  batch_size: 256
  num_workers: 0
  pin_memory: false
  drop_last: true
YML
TBAMD_CONFIG=$O/r50ex.yml TBAMD_EXAMPLE_MAX_ITERS=50 TBAMD_EXAMPLE_TIMING=20 timeout -k 10 500 python examples/img_cls/resnet/resnet.py > $O/r50ex.log 2>$O/r50ex.err; chk $? r50ex; grep example_img_s $O/r50ex.log
W="timeout -k 10 500 python scripts/bench_workloads.py"
for i in 1 2; do
$W --workload dcgan --mode native --steps 60 --warmup 10 > $O/dnat$i.log 2>$O/dnat$i.err; chk $? dnat$i; echo "dnat$i $(v dnat$i)"
TBAMD_CONV_SCHED=0 $W --workload dcgan --mode native --steps 60 --warmup 10 > $O/dnat0_$i.log 2>$O/dnat0_$i.err; chk $? dnat0_$i; echo "dnat0_$i $(v dnat0_$i)"
done
grep -h "host" $O/dnat1.err | tail -2
echo final rc=0
