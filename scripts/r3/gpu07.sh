#!/bin/bash
# native im2col/col2im convs + Gram backward + hardened tests; vendor-kernel census of the style / GAN examples
set -o pipefail
O=gpurun_out/r3_07; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_convgemm.py tests/test_gpu_gram.py tests/test_gpu_linear.py tests/test_gpu_r2_correctness.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export TBAMD_SYNTHETIC_DATA=1 TBAMD_EXAMPLE_MAX_ITERS=6 TBAMD_CONV_NO_MIOPEN=1 TBAMD_TUNE_LOG=1
printf "#include $GRAFT_REPO_ROOT/examples/img_gen/dcgan/dcgan.yml\nenv:\n  n_gpu: 1\n  fp16: true\n" > $O/dcgan1.yml
for ex in img_stt/offline/offline img_stt/online/online img_stt/adain/adain img_gen/dcgan/dcgan img_cls/lenet/lenet; do
  n=$(basename $ex)
  cfg=""; [ $n = dcgan ] && cfg="TBAMD_CONFIG=$GRAFT_REPO_ROOT/$O/dcgan1.yml"
  (cd $O && env $cfg timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d prof_$n -o $n -- python $GRAFT_REPO_ROOT/examples/$ex.py > $n.log 2>&1)
  chk $? $n
done
python scripts/vendor_kernels.py $(find $O -name "*_kernel_trace.csv") > $O/vendor.txt; cat $O/vendor.txt | grep -v "^  .*aten" | head -60
grep -h "conv-tune" $O/*.log | sort | uniq > $O/conv_tune.txt; wc -l $O/conv_tune.txt
