"""Small example models of the reference (MLP GAN / VAE, LeNet) on fused MI355X ops.

* LeNet — /root/reference/examples/img_cls/lenet/lenet.py:29-36 (conv5 -> BN ->
  GELU -> maxpool x2, MLP 256->120->84->10; 44,470 params).  BN+GELU is one fused
  NHWC kernel (:class:`BatchNormAct2d` act="gelu").
* MLP GAN Generator / Discriminator — examples/img_gen/gan/gan.py:31-49
  (730,896 / 665,089 params).  The discriminator stays on differentiable-twice
  ATen ops because the gradient penalty back-propagates through its gradient
  (SURVEY.md K23).
* VAE — examples/img_gen/vae/vae.py:29-70 (1,526,800 params).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor, nn

from torchbooster_amd.ops.norm import BatchNormAct2d
from torchbooster_amd.ops.linear import Linear

__all__ = ["LeNet", "lenet", "MLPGenerator", "MLPDiscriminator", "VAE", "VAEEncoder", "VAEDecoder"]


class LeNet(nn.Module):
    def __init__(self, num_classes: int = 10, in_ch: int = 1) -> None:
        super().__init__()
        self.c1 = nn.Conv2d(in_ch, 6, 5)
        self.n1 = BatchNormAct2d(6, act="gelu")
        self.c2 = nn.Conv2d(6, 16, 5)
        self.n2 = BatchNormAct2d(16, act="gelu")
        self.pool = nn.MaxPool2d(2)
        self.head = nn.Sequential(nn.Flatten(), Linear(256, 120), nn.GELU(), Linear(120, 84), nn.GELU(),
                                  Linear(84, num_classes))

    def forward(self, x: Tensor) -> Tensor:
        x = self.pool(self.n1(self.c1(x)))
        x = self.pool(self.n2(self.c2(x)))
        # NCHW flatten order, as the reference's nn.Flatten on NCHW
        return self.head(x.contiguous())


def lenet(num_classes: int = 10) -> LeNet:
    return LeNet(num_classes)


class MLPGenerator(nn.Sequential):
    def __init__(self, z_dim: int = 128, out_shape=(1, 28, 28)) -> None:
        self.z_dim = z_dim
        n = 1
        for s in out_shape:
            n *= s
        super().__init__(Linear(z_dim, 512), nn.GELU(), Linear(512, 512), nn.GELU(), Linear(512, n),
                         nn.Sigmoid(), nn.Unflatten(1, tuple(out_shape)))


class MLPDiscriminator(nn.Sequential):
    def __init__(self, in_features: int = 784) -> None:
        super().__init__(nn.Flatten(), Linear(in_features, 512), nn.GELU(), Linear(512, 512), nn.GELU(),
                         Linear(512, 1))


class VAEEncoder(nn.Sequential):
    def __init__(self, z_dim: int = 128, in_features: int = 784) -> None:
        self.z_dim = z_dim
        super().__init__(nn.Flatten(), Linear(in_features, 512), nn.GELU(), Linear(512, 512), nn.GELU(),
                         Linear(512, 2 * z_dim))

    def forward(self, x: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        h = super().forward(x)
        mu, log_var = torch.split(h, self.z_dim, dim=1)
        z = mu + torch.exp(0.5 * log_var) * torch.randn_like(log_var)
        return z, mu, log_var


class VAEDecoder(MLPGenerator):
    pass


class VAE(nn.Module):
    def __init__(self, z_dim: int = 128) -> None:
        super().__init__()
        self.z_dim = z_dim
        self.encoder = VAEEncoder(z_dim)
        self.decoder = VAEDecoder(z_dim)

    def forward(self, x: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        z, mu, log_var = self.encoder(x)
        return self.decoder(z), mu, log_var
