"""Hinge GAN with gradient penalty on MNIST (reference: examples/img_gen/gan/gan.py).

Same loop order as the reference (two D forwards before the two ``utils.step``
calls, GP through a double backward).  Under DDP the native reducer reduces
every backward pass and finalizes leftovers at the end of each backward, so the
discriminator's gradients stay rank-identical (the reference's torch-DDP version
silently desynchronised them — SURVEY.md A.2 B10).  The GP interpolation uses
``alpha*real + (1-alpha)*fake`` (the reference's minus sign, B12, is fixed) and
``sample`` handles the DDP wrapper (B13).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[3]))

import torch  # noqa: E402
from torch import Tensor, autograd  # noqa: E402
from torch.nn import Module  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
import torchbooster_amd.utils as utils  # noqa: E402
from torchbooster_amd.imageio import save_image  # noqa: E402
from common import max_iters, model_dtype, prepare_model, to_input  # noqa: E402
from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,  # noqa: E402
                                     OptimizerConfig, SchedulerConfig)
from torchbooster_amd.dataset import Split  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.models import MLPDiscriminator, MLPGenerator  # noqa: E402
from torchbooster_amd.ops.losses import hinge  # noqa: E402


def grad_penalty(D: Module, X_real: Tensor, X_fake: Tensor) -> Tensor:
    alpha = torch.rand((X_real.size(0),) + (1,) * (X_real.dim() - 1), device=X_real.device, dtype=X_real.dtype)
    t = (alpha * X_real + (1 - alpha) * X_fake).requires_grad_(True)
    Dt = D(t)
    grads = autograd.grad(Dt, t, torch.ones_like(Dt), create_graph=True, retain_graph=True)[0]
    return torch.mean((grads.view(grads.size(0), -1).float().norm(2, dim=1) - 1) ** 2)


@dataclass
class Config(BaseConfig):
    epochs: int
    seed: int
    z_dim: int
    grad_penalty: float

    env: EnvironementConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    dataset: DatasetConfig
    samples: str = "gan_samples.png"


def fit(conf, G, D, G_optim, G_sched, D_optim, D_sched, loader) -> None:
    limit = max_iters(len(loader))
    for epoch in range(conf.epochs if limit == len(loader) else 1):
        G.train()
        D.train()
        run_g, run_d = RunningAverage(), RunningAverage()
        for it, (X_real, _) in enumerate(loader):
            if it >= limit:
                break
            X_real = 1.0 - to_input(X_real, conf, channels_last=False)
            z = torch.randn((X_real.size(0), conf.z_dim), device=X_real.device, dtype=X_real.dtype)
            X_fake = G(z)
            with utils.frozen(D):  # the G step neither computes nor all-reduces D's gradient
                G_loss = hinge(D(X_fake), 1.0, -1.0)  # relu(1 - D(G(z))).mean()
            X_fake = utils.detach(X_fake)
            D_loss = hinge(D(X_real), 1.0, -1.0) + hinge(D(X_fake), 1.0, 1.0)
            D_loss = D_loss + conf.grad_penalty * grad_penalty(D, X_real, X_fake)
            utils.step(G_loss, G_optim, scheduler=G_sched)
            utils.step(D_loss, D_optim, scheduler=D_sched)
            run_g.update(G_loss.detach())
            run_d.update(D_loss.detach())
        if dist.is_primary():
            print(f"epoch {epoch} G_loss {run_g.value:.3e} D_loss {run_d.value:.3e}", flush=True)


def sample(conf, G) -> Tensor:
    G = getattr(G, "module", G)
    G.eval()
    with torch.no_grad():
        p = next(G.parameters())
        z = torch.randn((16 * 16, conf.z_dim), device=p.device, dtype=p.dtype)
        return 1.0 - G(z)


def main(conf: Config) -> None:
    data = conf.dataset.make(Split.TRAIN)
    loader = conf.loader.make(data, shuffle=True, distributed=conf.env.distributed)
    G = prepare_model(MLPGenerator(conf.z_dim), conf, channels_last=False)
    D = prepare_model(MLPDiscriminator(), conf, channels_last=False)
    G_optim = conf.optim.make(G.parameters())
    G_sched = conf.scheduler.make(G_optim)
    D_optim = conf.optim.make(D.parameters())
    D_sched = conf.scheduler.make(D_optim)
    fit(conf, G, D, G_optim, G_sched, D_optim, D_sched, loader)
    if dist.is_primary():
        imgs = sample(conf, G)
        out = save_image(imgs.float().view(-1, 1, 28, 28), conf.samples, nrow=16)  # reference gan.py:131
        print("samples", tuple(imgs.shape), float(imgs.float().mean()), "->", out)


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("gan.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
