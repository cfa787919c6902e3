"""LeNet on MNIST (reference: examples/img_cls/lenet/lenet.py).

Same Config / fit structure; BN+GELU is one fused kernel, cross-entropy and the
batch accuracy come out of one fused kernel, the running averages stay on the
device (no per-iteration host syncs).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[3]))

import torch  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
import torchbooster_amd.utils as utils  # noqa: E402
from common import max_iters, prepare_model, to_input  # noqa: E402
from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,  # noqa: E402
                                     OptimizerConfig, SchedulerConfig)
from torchbooster_amd.dataset import Split  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.models import lenet  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402


@dataclass
class Config(BaseConfig):
    epochs: int
    seed: int

    env: EnvironementConfig
    dataset: DatasetConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig


def run_epoch(conf, model, optim, scheduler, loader, train: bool, limit: int) -> dict:
    model.train(train)
    loss_avg, acc_avg = RunningAverage(), RunningAverage()
    for it, (X, labels) in enumerate(loader):
        if it >= limit:
            break
        X, labels = to_input(X, conf), conf.env.make(labels)
        with torch.set_grad_enabled(train):
            loss, acc = cross_entropy_accuracy(model(X), labels)
        if train:
            utils.step(loss, optim, scheduler)
        loss_avg.update(loss.detach())
        acc_avg.update(acc)
    return {"loss": loss_avg.value, "acc": acc_avg.value}


def main(conf: Config) -> None:
    train_set = conf.dataset.make(Split.TRAIN)
    test_set = conf.dataset.make(Split.TEST)
    train_loader = conf.loader.make(train_set, shuffle=True, distributed=conf.env.distributed)
    test_loader = conf.loader.make(test_set, shuffle=False, distributed=False)
    model = prepare_model(lenet(10), conf)
    optim = conf.optim.make(model.parameters())
    scheduler = conf.scheduler.make(optim)
    limit = max_iters(len(train_loader))
    for epoch in range(conf.epochs if limit == len(train_loader) else 1):
        stats = run_epoch(conf, model, optim, scheduler, train_loader, True, limit)
        if dist.is_primary():
            print(f"epoch {epoch} train {stats}", flush=True)
    if dist.is_primary():
        print("test", run_epoch(conf, model, optim, scheduler, test_loader, False, max_iters(len(test_loader))))


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("lenet.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
