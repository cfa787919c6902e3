"""ViT-B/16 training from LMDB with the native input pipeline (north-star config 5).

Records (uint8 HWC image + int64 label) are gathered from the LMDB file by the
native reader straight into pinned host buffers (C++ threads, no GIL), copied
H2D on a side HIP stream and crop/flip/normalised to bf16 NHWC on the device
(:class:`~torchbooster_amd.data.PinnedPrefetcher`).  Cosine CycleScheduler,
fused AdamW + clip, native DDP over RCCL.  Not in the reference (no attention
models there).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
import torchbooster_amd.utils as utils  # noqa: E402
from common import report_sync, max_iters, prepare_model, to_input, use_gpu  # noqa: E402
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.config import BaseConfig, EnvironementConfig, LoaderConfig, OptimizerConfig, SchedulerConfig  # noqa: E402
from torchbooster_amd.data import LMDBImageDataset, PinnedPrefetcher  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402


@dataclass
class Config(BaseConfig):
    epochs: int
    seed: int
    arch: str
    image: int
    num_classes: int
    clip: float
    label_smoothing: float
    lmdb: str
    lmdb_records: int
    prefetch_depth: int
    env: EnvironementConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig


def prepare(conf: Config) -> None:
    if os.path.exists(os.path.join(conf.lmdb, "data.mdb")):
        return
    g = np.random.default_rng(conf.seed)
    s = conf.image + 32  # room for random crops
    imgs = g.integers(0, 256, size=(conf.lmdb_records, s, s, 3), dtype=np.uint8)
    labels = g.integers(0, conf.num_classes, size=conf.lmdb_records)
    LMDBImageDataset.prepare(conf.lmdb, imgs, labels)


def main(conf: Config) -> None:
    if dist.is_primary():
        prepare(conf)
    dist.synchronize()
    ds = LMDBImageDataset(conf.lmdb)
    model = prepare_model(getattr(models, conf.arch)(num_classes=conf.num_classes, image=conf.image), conf,
                          channels_last=True)
    optim = conf.optim.make(model.parameters())
    sched = conf.scheduler.make(optim)
    if use_gpu(conf):
        loader = PinnedPrefetcher(ds, conf.loader.batch_size, depth=conf.prefetch_depth, seed=conf.seed,
                                  crop=(conf.image, conf.image), random_flip=True, rank=dist.get_rank(),
                                  world_size=dist.get_world_size())
    else:  # CPU plumbing: plain DataLoader over the same LMDB
        loader = conf.loader.make(ds, shuffle=True, distributed=conf.env.distributed)
    limit = max_iters(len(loader))
    for epoch in range(conf.epochs if limit == len(loader) else 1):
        if hasattr(loader, "set_epoch"):
            loader.set_epoch(epoch)
        run_loss, run_acc = RunningAverage(), RunningAverage()
        for it, (x, y) in enumerate(loader):
            if it >= limit:
                break
            if not use_gpu(conf):
                x = torch.nn.functional.interpolate(x, size=(conf.image, conf.image))
            x, y = to_input(x, conf), conf.env.make(y)
            loss, acc = cross_entropy_accuracy(model(x), y, conf.label_smoothing)
            utils.step(loss, optim, sched, clip=conf.clip)
            run_loss.update(loss.detach())
            run_acc.update(acc)
        if dist.is_primary():
            print(f"epoch {epoch} loss {run_loss.value:.4f} acc {run_acc.value:.4f}", flush=True)
    report_sync(model)


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("vit.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
