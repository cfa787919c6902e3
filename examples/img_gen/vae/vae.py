"""VAE on MNIST (reference: examples/img_gen/vae/vae.py).

Reconstruction loss is binary cross-entropy on the decoder's Sigmoid output.
(The reference applied ``binary_cross_entropy_with_logits`` to that Sigmoid
output — a double sigmoid; ``reference_double_sigmoid: true``
reproduces it.)
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
from common import max_iters, prepare_model, to_input  # noqa: E402
from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,  # noqa: E402
                                     OptimizerConfig, SchedulerConfig)
from torchbooster_amd.dataset import Split  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.models import VAE  # noqa: E402
from torchbooster_amd.ops.losses import bce_with_logits, gaussian_kld  # noqa: E402


@dataclass
class Config(BaseConfig):
    epochs: int
    seed: int
    z_dim: int
    kld_weight: float
    clip: float

    env: EnvironementConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    dataset: DatasetConfig
    reference_double_sigmoid: bool = False
    samples: str = "vae_samples.png"


def kld(mu, log_var):
    """mean_b(-0.5 Σ (1 + log_var - mu² - exp(log_var))) — vae.py:72-75 (fused K21 kernel on GPU)."""
    return gaussian_kld(mu, log_var)


def main(conf: Config) -> None:
    data = conf.dataset.make(Split.TRAIN)
    loader = conf.loader.make(data, shuffle=True, distributed=conf.env.distributed)
    vae = prepare_model(VAE(conf.z_dim), conf, channels_last=False)
    optim = conf.optim.make(vae.parameters())
    sched = conf.scheduler.make(optim)
    limit = max_iters(len(loader))
    for epoch in range(conf.epochs if limit == len(loader) else 1):
        vae.train()
        run = RunningAverage()
        for it, (X, _) in enumerate(loader):
            if it >= limit:
                break
            X = to_input(X, conf, channels_last=False)
            X_rec, mu, log_var = vae(X)
            if conf.reference_double_sigmoid:
                rec = bce_with_logits(X_rec, X)
            else:
                rec = F.binary_cross_entropy(X_rec.float().clamp(1e-6, 1 - 1e-6), X.float())
            loss = rec + conf.kld_weight * kld(mu, log_var)
            utils.step(loss, optim, scheduler=sched, clip=conf.clip)
            run.update(loss.detach())
        if dist.is_primary():
            print(f"epoch {epoch} loss {run.value:.4e}", flush=True)
    if dist.is_primary():
        out = save_image(sample(conf, vae).float().view(-1, 1, 28, 28), conf.samples, nrow=16)
        print("samples ->", out)


def sample(conf: Config, vae) -> torch.Tensor:
    """16 x 16 decoded draws from the prior, shown inverted like the reference (vae.py:127-135)."""
    dec = getattr(vae, "module", vae).decoder
    dec.eval()
    with torch.no_grad():
        p = next(dec.parameters())
        z = torch.randn((16 * 16, conf.z_dim), device=p.device, dtype=p.dtype)
        return 1.0 - dec(z)


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("vae.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
