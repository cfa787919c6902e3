#!/bin/bash
set -o pipefail
O=gpurun_out/r3_11; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
export TBAMD_SYNTHETIC_DATA=1 TBAMD_EXAMPLE_MAX_ITERS=6 TBAMD_CONV_NO_MIOPEN=1
for ex in img_cls/lenet/lenet img_gen/gan/gan; do
  n=$(basename $ex)
  timeout -k 10 240 python scripts/r3/blas_spy.py examples/$ex.py > $O/$n.out 2> $O/$n.err; chk $? $n
  grep blas-spy $O/$n.err | head -30
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_trajectory.py tests/test_gpu_ddp.py tests/test_gpu_convgemm.py tests/test_gpu_gram.py tests/test_gpu_linear.py tests/test_gpu_r2_correctness.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export TBAMD_TUNE_LOG=1
unset TBAMD_CONV_NO_MIOPEN
printf "#include $GRAFT_REPO_ROOT/examples/img_gen/dcgan/dcgan.yml\nenv:\n  n_gpu: 1\n  fp16: true\nloader:\n  batch_size: 128\n  num_workers: 0\n  pin_memory: true\n  drop_last: true\n" > $O/dcgan1.yml
for ex in img_gen/dcgan/dcgan img_stt/online/online; do
  n=$(basename $ex)
  cfg=""; [ $n = dcgan ] && cfg="TBAMD_CONFIG=$GRAFT_REPO_ROOT/$O/dcgan1.yml"
  (cd $O && env $cfg timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d prof_$n -o $n -- python $GRAFT_REPO_ROOT/examples/$ex.py > $n.log 2>&1)
  chk $? $n
done
python scripts/vendor_kernels.py $(find $O -name "*_kernel_trace.csv") > $O/vendor.txt; grep -v "^  .*aten" $O/vendor.txt | head -40
grep -h "conv-tune" $O/*.log | sort | uniq > $O/conv_tune.txt; cat $O/conv_tune.txt
