"""Style-transfer models and losses (examples/img_stt of the reference).

* :class:`StyleNet` — Johnson et al. feed-forward net, /root/reference/examples/img_stt/online/online.py:37-57
  (ReflectionPad + Conv + InstanceNorm(affine) + GELU blocks; the five residual
  bottlenecks are ONE weight-tied module, 496,515 params — SURVEY.md A.2 B19).
* :class:`AdaINDecoder` + :func:`adain` / :func:`mu_std` — adain.py:36-63
  (2,931,267 params).
* :func:`gram_matrix` / :func:`total_variation` — online.py:60-69, offline.py:25-34.

InstanceNorm + GELU runs as one fused NHWC GroupNorm kernel
(:class:`~torchbooster_amd.ops.norm.InstanceNormAct2d`, G = C).  The Gram
matrix is computed from the channels_last layout directly without the NCHW
transpose copy: on the native split-K SYRK kernel (ops/gram.py,
csrc/gram.hip) for bf16 features, one batched GEMM (K = H*W) otherwise.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops.conv import Conv2d
from torchbooster_amd.ops.gram import gram
from torchbooster_amd.ops.gram import native_f32_supported as gram_native_f32_supported
from torchbooster_amd.ops.gram import native_supported as gram_native_supported

from torchbooster_amd.ops.losses import mean_std
from torchbooster_amd.ops.losses import style_stats_loss
from torchbooster_amd.ops.losses import total_variation as _tv
from torchbooster_amd.ops.norm import InstanceNormAct2d
from torchbooster_amd.ops.resample import ReflectionPad2d, UpsampleNearest2d

__all__ = ["conv_pad", "ConvIN", "DeconvIN", "Bottleneck", "Residual", "StyleNet", "AdaINDecoder", "gram_matrix",
           "gram_matrix_flat", "total_variation", "mu_std", "adain", "style_stats_loss"]


class PadConv(nn.Sequential):
    """ReflectionPad2d(k//2) + Conv2d — the reference's ``Conv`` lambda (same module
    tree / state-dict keys), run as ONE conv whose reflect padding is folded into the
    kernel's input addressing (csrc/conv_any.hip; ops.conv.conv2d_any)."""

    def __init__(self, i: int, o: int, k: int, s: int) -> None:
        super().__init__(ReflectionPad2d(k // 2), Conv2d(i, o, k, s))
        self.fold = (k // 2, True, 1)

    def forward(self, x: Tensor) -> Tensor:
        return self[1](x, fold=self.fold)


def conv_pad(i: int, o: int, k: int, s: int) -> nn.Sequential:
    """ReflectionPad2d(k//2) + Conv2d — the reference's ``Conv`` lambda."""
    return PadConv(i, o, k, s)


class ConvIN(nn.Sequential):
    """Conv -> InstanceNorm(affine) -> GELU (norm + GELU fused)."""

    def __init__(self, i: int, o: int, k: int, s: int) -> None:
        super().__init__(conv_pad(i, o, k, s), InstanceNormAct2d(o, act="gelu"))


class DeconvIN(nn.Sequential):
    """Upsample x2 -> ConvIN -> GELU (the reference applies GELU twice).  The
    nearest upsampling is folded into the conv's addressing with the reflect
    padding: no 4x-sized intermediate is written."""

    def __init__(self, i: int, o: int, k: int, s: int) -> None:
        super().__init__(UpsampleNearest2d(scale_factor=2), ConvIN(i, o, k, s), nn.GELU())
        self.fold = (k // 2, True, 2)

    def forward(self, x: Tensor) -> Tensor:
        ci = self[1]
        return self[2](ci[1](ci[0][1](x, fold=self.fold)))


class Bottleneck(nn.Sequential):
    def __init__(self, i: int, o: int, k: int, s: int) -> None:
        super().__init__(ConvIN(i, o, k, s), nn.GELU(), ConvIN(o, i, k, s))


class Residual(nn.Module):
    def __init__(self, *modules: nn.Module) -> None:
        super().__init__()
        self.module = nn.Sequential(*modules)

    def forward(self, x: Tensor) -> Tensor:
        return x + self.module(x)


class StyleNet(nn.Sequential):
    def __init__(self) -> None:
        res = Residual(Bottleneck(128, 128, 3, 1))
        inner = nn.Sequential(ConvIN(64, 128, 3, 2), *([res] * 5), DeconvIN(128, 64, 3, 1))
        mid = nn.Sequential(ConvIN(32, 64, 3, 2), inner, DeconvIN(64, 32, 3, 1))
        super().__init__(ConvIN(3, 32, 9, 1), mid, conv_pad(32, 3, 9, 1))


class AdaINDecoder(nn.Sequential):
    def __init__(self) -> None:
        super().__init__(
            ConvIN(512, 256, 3, 1), DeconvIN(256, 256, 3, 1), ConvIN(256, 256, 3, 1), ConvIN(256, 128, 3, 1),
            DeconvIN(128, 128, 3, 1), ConvIN(128, 64, 3, 1), DeconvIN(64, 64, 3, 1), conv_pad(64, 3, 9, 1))


def gram_matrix(features: Tensor) -> Tensor:
    """Per-sample Gram ``F F^T / (C H W)`` -> [B, C, C] f32 (online.py:60-63).

    bf16 channels_last features with C % 64 == 0 run on the native split-K SYRK
    kernel (ops/gram.py); others use one batched GEMM."""
    B, C, H, W = features.shape
    if gram_native_supported(features) or gram_native_f32_supported(features):
        return gram(features, 1.0 / (C * H * W))
    if features.is_contiguous(memory_format=torch.channels_last) and not features.is_contiguous():
        f = features.permute(0, 2, 3, 1).reshape(B, H * W, C)  # [B, HW, C], free view of NHWC
        return torch.bmm(f.transpose(1, 2), f) / (C * H * W)
    f = features.reshape(B, C, H * W)
    return torch.bmm(f, f.transpose(1, 2)) / (C * H * W)


def gram_matrix_flat(features: Tensor) -> Tensor:
    """Whole-batch Gram ``F F^T / (B C H W)`` with F = features.view(-1, HW) (offline.py:25-28)."""
    B, C, H, W = features.shape
    if B == 1 and (gram_native_supported(features) or gram_native_f32_supported(features)):
        return gram(features, 1.0 / (C * H * W))[0]
    if features.is_contiguous(memory_format=torch.channels_last) and not features.is_contiguous() and B == 1:
        f = features.permute(0, 2, 3, 1).reshape(H * W, C)
        return (f.t() @ f) / (B * C * H * W)
    f = features.reshape(-1, H * W)
    return (f @ f.t()) / (B * C * H * W)


def total_variation(x: Tensor) -> Tensor:
    """Σ|x[..., w] - x[..., w+1]| + Σ|x[h] - x[h+1]| (K19 kernel on GPU, ops/losses.py)."""
    return _tv(x)


def mu_std(feat: Tensor, eps: float = 1e-5) -> Tuple[Tensor, Tensor]:
    """Per-(n, c) mean / sqrt(unbiased var + eps), expanded to ``feat`` (K20 kernel on GPU)."""
    mu, std = mean_std(feat, eps)
    mu = mu.to(feat.dtype)[:, :, None, None]
    std = std.to(feat.dtype)[:, :, None, None]
    return mu.expand_as(feat), std.expand_as(feat)


def adain(s_feat: Tensor, c_feat: Tensor) -> Tensor:
    (s_mu, s_std), (c_mu, c_std) = mu_std(s_feat), mu_std(c_feat)
    return s_std * (c_feat - c_mu) / c_std + s_mu
