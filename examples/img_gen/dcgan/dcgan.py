"""DCGAN 128x128 (north-star config 3; not in the reference, whose GAN is an MLP).

Non-saturating GAN loss, generator and discriminator each stepped by
``utils.step`` with their own optimizer/scheduler; the generator step runs D
under ``utils.frozen`` (no D weight gradients, no D all-reduce under DDP); a
sample grid is written to ``samples`` at the end; checkpoints through
``SaveCallback``.  BN+ReLU / BN+LeakyReLU are fused native kernels; images
are resized 224->128 by average pooling of the synthetic ImageNet-shape data
(offline environment).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[3]))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
import torchbooster_amd.utils as utils  # noqa: E402
from torchbooster_amd.imageio import save_image  # noqa: E402
from common import report_sync, max_iters, prepare_model, to_input  # noqa: E402
from torchbooster_amd.callbacks import SaveCallback  # noqa: E402
from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,  # noqa: E402
                                     OptimizerConfig, SchedulerConfig)
from torchbooster_amd.dataset import Split  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.models import DCGANDiscriminator, DCGANGenerator  # noqa: E402


@dataclass
class Config(BaseConfig):
    epochs: int
    seed: int
    z_dim: int
    width: int
    image: int

    env: EnvironementConfig
    dataset: DatasetConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    ckpt_every: int = 0
    ckpt_dir: str = "/tmp/dcgan_ckpt"
    samples: str = "dcgan_samples.png"


def main(conf: Config) -> None:
    data = conf.dataset.make(Split.TRAIN)
    loader = conf.loader.make(data, shuffle=True, distributed=conf.env.distributed)
    G = prepare_model(DCGANGenerator(conf.z_dim, conf.width), conf)
    D = prepare_model(DCGANDiscriminator(conf.width), conf)
    G_optim, D_optim = conf.optim.make(G.parameters()), conf.optim.make(D.parameters())
    G_sched, D_sched = conf.scheduler.make(G_optim), conf.scheduler.make(D_optim)
    saver = SaveCallback(conf.ckpt_every, conf.scheduler.n_iter, Path(conf.ckpt_dir), "dcgan") \
        if conf.ckpt_every > 0 else None
    limit = max_iters(len(loader))
    for epoch in range(conf.epochs if limit == len(loader) else 1):
        run_g, run_d = RunningAverage(), RunningAverage()
        for it, (X, _) in enumerate(loader):
            if it >= limit:
                break
            X = to_input(X, conf)
            if X.shape[-1] != conf.image:
                X = F.adaptive_avg_pool2d(X, conf.image)
            X = X * 2 - 1
            z = torch.randn(X.shape[0], conf.z_dim, device=X.device, dtype=X.dtype)
            fake = G(z)
            d_loss = F.softplus(-D(X)).float().mean() + F.softplus(D(fake.detach())).float().mean()
            utils.step(d_loss, D_optim, scheduler=D_sched)
            with utils.frozen(D):  # G step: no D weight gradients, no D all-reduce
                g_loss = F.softplus(-D(fake)).float().mean()
            utils.step(g_loss, G_optim, scheduler=G_sched)
            run_g.update(g_loss.detach())
            run_d.update(d_loss.detach())
            if saver is not None:
                saver(G=G, D=D, G_optim=G_optim, D_optim=D_optim, G_sched=G_sched, D_sched=D_sched)
        if dist.is_primary():
            print(f"epoch {epoch} G {run_g.value:.3e} D {run_d.value:.3e}", flush=True)
    report_sync(G, D)
    if dist.is_primary():
        g = getattr(G, "module", G)
        g.eval()
        with torch.no_grad():
            p = next(g.parameters())
            imgs = g(torch.randn(64, conf.z_dim, device=p.device, dtype=p.dtype)).float() * 0.5 + 0.5
        print("samples ->", save_image(imgs, conf.samples, nrow=8))


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("dcgan.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
