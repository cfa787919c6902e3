"""ResNet image classification (reference: examples/img_cls/resnet/resnet.py).

ResNet-18 on CIFAR-10 by default (``resnet.yml``, the reference's config) or
ResNet-50 ImageNet-shape over every GPU (``resnet50_imagenet.yml``).  The model
runs channels_last bf16 with f32 master weights in the fused AdamW; conv+BN
statistics, BN+ReLU(+residual), cross-entropy+accuracy, clip+AdamW are native
kernels; DDP is the native bucketed RCCL reducer.  torchvision's pretrained
weights are not available offline: random init.
"""
from __future__ import annotations

import json
import os
import sys
import time
from dataclasses import dataclass
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[3]))

import torch  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
import torchbooster_amd.utils as utils  # noqa: E402
from common import max_iters, prepare_model, to_input  # noqa: E402
from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.callbacks import SaveCallback  # noqa: E402
from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,  # noqa: E402
                                     OptimizerConfig, SchedulerConfig)
from torchbooster_amd.dataset import Split  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402


@dataclass
class Config(BaseConfig):
    epochs: int
    seed: int
    clip: float
    label_smoothing: float

    env: EnvironementConfig
    dataset: DatasetConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    arch: str = "resnet18"
    num_classes: int = 10
    ckpt_dir: str = ""
    ckpt_every: int = 0


def step(conf, model, optim, scheduler, loader, train: bool, limit: int, saver=None):
    model.train(train)
    run_loss, run_acc = RunningAverage(), RunningAverage()
    # TBAMD_EXAMPLE_TIMING=W: training throughput over the iterations after the first W (synchronised
    # on both sides, every rank's global batch), printed as one JSON line -- the figure bench.py's
    # headline number is checked against
    warm = int(os.environ.get("TBAMD_EXAMPLE_TIMING", "0")) if train else 0
    t0, n_timed, n_img = None, 0, 0
    for it, (X, labels) in enumerate(loader):
        if it >= limit:
            break
        if warm and it == warm and torch.cuda.is_available():
            dist.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        if t0 is not None:
            n_timed += 1
            n_img += X.shape[0]
        X, labels = to_input(X, conf), conf.env.make(labels)
        with torch.set_grad_enabled(train):
            loss, acc = cross_entropy_accuracy(model(X), labels, conf.label_smoothing)
        if train:
            utils.step(loss, optim, scheduler=scheduler, clip=conf.clip)
            if saver is not None:
                saver(model=model, optim=optim, scheduler=scheduler)
        run_loss.update(loss.detach())
        run_acc.update(acc)
    if t0 is not None and n_timed:
        torch.cuda.synchronize()
        dist.synchronize()
        dt = time.perf_counter() - t0
        if dist.is_primary():
            print(json.dumps({"example_img_s": round(n_img * dist.get_world_size() / dt, 2), "iters": n_timed,
                              "ms_per_iter": round(dt / n_timed * 1e3, 3)}), flush=True)
    return {"loss": run_loss.value, "acc": run_acc.value}


# the reference's CIFAR-10 transforms (examples/img_cls/resnet/resnet.py:92-106): on a GPU
# the whole pipeline runs in one kernel per batch over the HBM-resident uint8 dataset
CIFAR_MEAN, CIFAR_STD = (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)


def transforms(conf: Config):
    from torchbooster_amd.data import DeviceAugment

    if conf.num_classes != 10 and conf.num_classes != 100:  # ImageNet-shape runs: crop + flip only
        return DeviceAugment(hflip=True), DeviceAugment()
    train = DeviceAugment(size=32, padding=4, hflip=True, rotate=15, randaugment=True,
                          mean=CIFAR_MEAN, std=CIFAR_STD)
    return train, DeviceAugment(mean=CIFAR_MEAN, std=CIFAR_STD)


def main(conf: Config) -> None:
    train_tf, test_tf = transforms(conf)
    train_set = conf.dataset.make(Split.TRAIN, transform=train_tf)
    test_set = conf.dataset.make(Split.TEST, transform=test_tf)
    train_loader = conf.loader.make(train_set, shuffle=True, distributed=conf.env.distributed)
    test_loader = conf.loader.make(test_set, shuffle=False, distributed=False)
    model = prepare_model(getattr(models, conf.arch)(num_classes=conf.num_classes), conf)
    optim = conf.optim.make(model.parameters())
    scheduler = conf.scheduler.make(optim)
    saver = None
    if conf.ckpt_dir and conf.ckpt_every > 0:
        saver = SaveCallback(conf.ckpt_every, conf.scheduler.n_iter, Path(conf.ckpt_dir), conf.arch)
    limit = max_iters(len(train_loader))
    epochs = conf.epochs if limit == len(train_loader) else 1
    for epoch in range(epochs):
        if hasattr(train_loader.sampler, "set_epoch"):
            train_loader.sampler.set_epoch(epoch)
        stats = step(conf, model, optim, scheduler, train_loader, True, limit, saver)
        if dist.is_primary():
            print(f"epoch {epoch} train {stats}", flush=True)
    if dist.is_primary():
        print("test", step(conf, model, optim, scheduler, test_loader, False, max_iters(len(test_loader))))


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("resnet.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
