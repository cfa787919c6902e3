"""DCGAN at 128x128 (BASELINE.json config 3: "DCGAN 128x128 bf16 on 4xMI355X").

Not in the reference (its GAN is an MLP on 28x28 MNIST, gan.py:31-49; see
:mod:`torchbooster_amd.models.small`).  Standard Radford et al. layout scaled to
128 px: the generator is five stride-2 ConvTranspose 4x4 up-samplings from a
4x4x1024 seed with fused BN+ReLU, the discriminator five stride-2 Conv 4x4
down-samplings with fused BN+LeakyReLU(0.2).
"""
from __future__ import annotations

from torch import Tensor, nn

from torchbooster_amd.ops.act import LeakyReLU
from torchbooster_amd.ops.conv import Conv2d, ConvTranspose2d
from torchbooster_amd.ops.norm import BatchNormAct2d

__all__ = ["DCGANGenerator", "DCGANDiscriminator", "dcgan128"]


class _UpBlock(nn.Module):
    def __init__(self, i: int, o: int, first: bool = False) -> None:
        super().__init__()
        self.conv = ConvTranspose2d(i, o, 4, 1 if first else 2, 0 if first else 1, bias=False)  # native (K27)
        self.bn = BatchNormAct2d(o, act="relu")

    def forward(self, x: Tensor) -> Tensor:
        return self.bn(self.conv(x))


class _DownBlock(nn.Module):
    def __init__(self, i: int, o: int, norm: bool = True) -> None:
        super().__init__()
        self.conv = Conv2d(i, o, 4, 2, 1, bias=not norm)  # native (3-channel input: generic family), autotuned
        self.bn = BatchNormAct2d(o, act="leaky_relu", slope=0.2) if norm else None
        self.act = None if norm else LeakyReLU(0.2)  # native elementwise kernels (ops/act.py)

    def forward(self, x: Tensor) -> Tensor:
        x = self.conv(x)
        return self.bn(x) if self.bn is not None else self.act(x)


class DCGANGenerator(nn.Module):
    def __init__(self, z_dim: int = 128, width: int = 64, out_ch: int = 3) -> None:
        super().__init__()
        self.z_dim = z_dim
        w = width
        self.blocks = nn.Sequential(
            _UpBlock(z_dim, 16 * w, first=True),  # 4
            _UpBlock(16 * w, 8 * w),  # 8
            _UpBlock(8 * w, 4 * w),  # 16
            _UpBlock(4 * w, 2 * w),  # 32
            _UpBlock(2 * w, w),  # 64
        )
        self.out = ConvTranspose2d(w, out_ch, 4, 2, 1)  # 128 (3 outputs: the generic conv family)
        self.tanh = nn.Tanh()

    def forward(self, z: Tensor) -> Tensor:
        return self.tanh(self.out(self.blocks(z.view(z.shape[0], self.z_dim, 1, 1))))


class DCGANDiscriminator(nn.Module):
    def __init__(self, width: int = 64, in_ch: int = 3) -> None:
        super().__init__()
        w = width
        self.blocks = nn.Sequential(
            _DownBlock(in_ch, w, norm=False),  # 64
            _DownBlock(w, 2 * w),  # 32
            _DownBlock(2 * w, 4 * w),  # 16
            _DownBlock(4 * w, 8 * w),  # 8
            _DownBlock(8 * w, 16 * w),  # 4
        )
        self.out = Conv2d(16 * w, 1, 4, 1, 0)  # 1 output channel: the generic conv family

    def forward(self, x: Tensor) -> Tensor:
        return self.out(self.blocks(x)).flatten(1)


def dcgan128(z_dim: int = 128, width: int = 64):
    return DCGANGenerator(z_dim, width), DCGANDiscriminator(width)
