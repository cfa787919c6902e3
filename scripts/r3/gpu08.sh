#!/bin/bash
# side-stream wgrad A/B + native conv/Gram tests + vendor-kernel census of the style / GAN examples
set -o pipefail
O=gpurun_out/r3_08; mkdir -p $O
chk() { rc=$1; echo "$2 rc=$rc"; [ $rc -eq 0 ] || tail -30 $O/$2.err; [ $rc -lt 124 ] || exit $rc; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_trajectory.py tests/test_gpu_ddp.py tests/test_gpu_convgemm.py tests/test_gpu_gram.py tests/test_gpu_linear.py tests/test_gpu_r2_correctness.py > $O/t.err 2>&1 ; chk $? t; tail -2 $O/t.err
for s in 0 1 0 1; do
  TBAMD_WGRAD_STREAM=$s timeout -k 10 200 python bench.py --steps 40 --warmup 15 > $O/bench_s$s.json 2> $O/bench.err; chk $? bench; cat $O/bench_s$s.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_r50 -o r50 -- python bench.py --steps 10 --warmup 10 > $O/prof_r50.log 2>&1; chk $? prof_r50
export TBAMD_SYNTHETIC_DATA=1 TBAMD_EXAMPLE_MAX_ITERS=6 TBAMD_CONV_NO_MIOPEN=1 TBAMD_TUNE_LOG=1
printf "#include $GRAFT_REPO_ROOT/examples/img_gen/dcgan/dcgan.yml\nenv:\n  n_gpu: 1\n  fp16: true\nloader:\n  num_workers: 0\n" > $O/dcgan1.yml
for ex in img_stt/offline/offline img_stt/online/online img_stt/adain/adain img_gen/dcgan/dcgan img_cls/lenet/lenet; do
  n=$(basename $ex)
  cfg=""; [ $n = dcgan ] && cfg="TBAMD_CONFIG=$GRAFT_REPO_ROOT/$O/dcgan1.yml"
  (cd $O && env $cfg timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d prof_$n -o $n -- python $GRAFT_REPO_ROOT/examples/$ex.py > $n.log 2>&1)
  chk $? $n
done
python scripts/vendor_kernels.py $(find $O -name "*_kernel_trace.csv" -path "*prof_[a-z]*" ! -path "*prof_r50*") > $O/vendor.txt; grep -v "^  .*aten" $O/vendor.txt | head -60
grep -h "conv-tune" $O/*.log | sort | uniq > $O/conv_tune.txt; wc -l $O/conv_tune.txt
