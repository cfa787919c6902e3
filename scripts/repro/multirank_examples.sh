#!/bin/bash
# Multi-rank rehearsals of the north-star example configs on the CPU (gloo), through the examples'
# own Config.load -> launch (torchrun env://) -> env.make (native DDP) -> utils.step pipeline, with
# the DDP desync self-check (TBAMD_DDP_CHECK=1: every rank's reduced gradients compared with rank
# 0's after each reduction) and a final cross-rank parameter comparison (TBAMD_REPORT_SYNC=1):
#   * DCGAN-128 (BASELINE config 3) at 4 ranks: the two-optimizer G/D step, D frozen for the G step
#   * ViT-B/16 224 px (config 5) at 8 ranks from torchbooster.lmdb through LoaderConfig, cycle
#     scheduler with cosine decay, AdamW + clip
# Throughput here measures nothing (CPU ranks); what is checked is that the multi-rank path runs
# and stays in sync.  Usage: bash scripts/repro/multirank_examples.sh OUT_DIR
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=${1:-/tmp/multirank}; mkdir -p $O
export CUDA_VISIBLE_DEVICES= HIP_VISIBLE_DEVICES= TBAMD_DDP_CHECK=1 TBAMD_REPORT_SYNC=1 OMP_NUM_THREADS=1
run() {  # name nproc script config-override
  n=$1; np=$2; script=$3; printf '%b' "$4" > $O/$n.yml
  TBAMD_CONFIG=$O/$n.yml timeout -k 10 1500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $((29700 + np)) $R/$script > $O/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; grep -E "^\[sync\]|^epoch" $O/$n.log; [ $rc -eq 0 ] || { tail -30 $O/$n.log; exit $rc; }
}
TBAMD_EXAMPLE_MAX_ITERS=3 TBAMD_SYNTHETIC_LEN=64 TBAMD_SYNTHETIC_DATA=1 run dcgan128_4rank 4 examples/img_gen/dcgan/dcgan.py \
  "#include $R/examples/img_gen/dcgan/dcgan.yml\nsamples: $O/dcgan_samples.png\nenv:\n  n_gpu: 4\n  distributed: true\nloader:\n  batch_size: 4\n  num_workers: 0\n  drop_last: true\n"
TBAMD_EXAMPLE_MAX_ITERS=2 run vitb16_8rank_lmdb 8 examples/vit/vit.py \
  "#include $R/examples/vit/vit.yml\nlmdb: $O/vit_lmdb\nlmdb_records: 64\nenv:\n  n_gpu: 8\n  distributed: true\nloader:\n  batch_size: 2\n  num_workers: 0\n  drop_last: true\n"
echo final rc=0
