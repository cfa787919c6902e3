"""Fused scalar losses and per-channel statistics of the generative / style examples.

One HIP kernel family (``csrc/aux_ops.hip``) per SURVEY.md §2.3.1 row:

* K19 :func:`total_variation` — Σ|∂x/∂w| + Σ|∂x/∂h|
  (/root/reference/examples/img_stt/online/online.py:66-69, offline.py:31-34);
* K20 :func:`mean_std` — per-(n, c) mean and unbiased std + eps of AdaIN
  (/root/reference/examples/img_stt/adain/adain.py:55-63);
* K21 :func:`bce_with_logits` and :func:`gaussian_kld` — the VAE losses
  (/root/reference/examples/img_gen/vae/vae.py:72-75,112);
* K22 :func:`hinge` — ``relu(margin + sign·D(x)).mean()`` of the hinge GAN
  (/root/reference/examples/img_gen/gan/gan.py:104,107).

Forward: a persistent grid writes per-workgroup partials, one workgroup folds
them in f64 (deterministic).  Backward reads the upstream gradient from device
memory, so none of these synchronise with the host and all are
hipGraph-capturable.  CPU tensors take the PyTorch expressions the reference
writes (they double as the numerics reference in the GPU tests).
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor
from torch.autograd.function import once_differentiable

from torchbooster_amd.ops._ext import native, use_native

__all__ = ["total_variation", "hinge", "bce_with_logits", "gaussian_kld", "mean_std", "style_stats_loss",
           "total_variation_ref", "hinge_ref", "gaussian_kld_ref", "mean_std_ref"]

_FLOATS = (torch.float32, torch.bfloat16, torch.float16)


def _layout_ok(x: Tensor) -> bool:
    return x.dim() == 4 and (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last))


# --------------------------------------------------------------- references
def total_variation_ref(x: Tensor) -> Tensor:
    a = (x[:, :, :, :-1] - x[:, :, :, 1:]).abs().sum()
    b = (x[:, :, :-1, :] - x[:, :, 1:, :]).abs().sum()
    return a + b


def hinge_ref(x: Tensor, margin: float = 1.0, sign: float = -1.0) -> Tensor:
    return torch.relu(margin + sign * x).float().mean()


def gaussian_kld_ref(mu: Tensor, log_var: Tensor) -> Tensor:
    mu, log_var = mu.float(), log_var.float()
    return torch.mean(-0.5 * torch.sum(1 + log_var - mu ** 2 - log_var.exp(), dim=1))


def mean_std_ref(x: Tensor, eps: float = 1e-5) -> Tuple[Tensor, Tensor]:
    mu = x.mean(dim=[2, 3])
    std = x.var(dim=[2, 3]).add(eps).sqrt()
    return mu, std


# ------------------------------------------------------------ autograd fns
class _TVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return native().tv_forward(x)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return native().tv_backward(x, g)


class _HingeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, margin, sign):
        ctx.save_for_backward(x)
        ctx.cfg = (margin, sign)
        return native().hinge_forward(x, margin, sign)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return native().hinge_backward(x, g, *ctx.cfg).view_as(x), None, None


class _BCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        ctx.save_for_backward(x, y)
        return native().bce_logits_forward(x, y)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        return native().bce_logits_backward(x, y, g).view_as(x), None


class _KLDFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, lv):
        ctx.save_for_backward(mu, lv)
        return native().kld_forward(mu, lv)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        mu, lv = ctx.saved_tensors
        dmu, dlv = native().kld_backward(mu, lv, g)
        return dmu, dlv.to(lv.dtype)


class _MeanStdFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eps):
        mean, std = native().mean_std_forward(x, eps)
        ctx.save_for_backward(x, mean, std)
        return mean, std

    @staticmethod
    @once_differentiable
    def backward(ctx, gmean, gstd):
        x, mean, std = ctx.saved_tensors
        if gmean is None:
            gmean = torch.zeros_like(mean)
        if gstd is None:
            gstd = torch.zeros_like(std)
        return native().mean_std_backward(x, mean, std, gmean, gstd), None


# ------------------------------------------------------------------ public
def total_variation(x: Tensor) -> Tensor:
    """Anisotropic total variation (sum of absolute neighbour differences), f32 scalar on GPU."""
    if use_native(x) and x.dtype in _FLOATS and _layout_ok(x) and x.size(2) > 0 and x.size(3) > 0:
        return _TVFn.apply(x)
    return total_variation_ref(x)


def hinge(x: Tensor, margin: float = 1.0, sign: float = -1.0) -> Tensor:
    """``relu(margin + sign * x).float().mean()``: sign=-1 → relu(1 - D), sign=+1 → relu(1 + D)."""
    if use_native(x) and x.dtype in _FLOATS and x.numel() > 0:
        return _HingeFn.apply(x, float(margin), float(sign))
    return hinge_ref(x, margin, sign)


def bce_with_logits(x: Tensor, target: Tensor) -> Tensor:
    """Mean binary cross-entropy on logits (numerically stable form), f32 scalar."""
    if use_native(x) and x.dtype in _FLOATS and x.numel() > 0 and target.shape == x.shape \
            and not target.requires_grad:
        return _BCEFn.apply(x, target)
    return F.binary_cross_entropy_with_logits(x.float(), target.float())


def gaussian_kld(mu: Tensor, log_var: Tensor) -> Tensor:
    """``mean_b(-0.5 Σ_d (1 + log_var - mu² - exp(log_var)))`` (the VAE's KL term)."""
    if use_native(mu) and mu.dtype in _FLOATS and mu.dim() == 2 and mu.shape == log_var.shape and mu.numel() > 0:
        return _KLDFn.apply(mu, log_var)
    return gaussian_kld_ref(mu, log_var)


def style_stats_loss(mixed: Sequence[Tensor], style: Sequence[Tensor], eps: float = 1e-5) -> Tensor:
    """AdaIN style loss ``Σ_l mse(μ(m_l), μ(s_l)) + mse(σ(m_l), σ(s_l))`` on per-(n, c) statistics.

    Equal to the reference's ``mse_loss`` over the spatially EXPANDED mean / std tensors
    (/root/reference/examples/img_stt/adain/adain.py:55-58 ``mu_std`` + :134 ``s_criterion``):
    every statistic is repeated H*W times, so the mean of the squared differences over the
    expansion is the mean over [N, C].  The [N, C, H, W] broadcasts (134 M elements at the
    relu1_2 hook of E7's b32 @256 step) and their gradients are never materialised; the
    statistics come from the native K20 kernel (f32) and its backward."""
    total: Optional[Tensor] = None
    for m, s in zip(mixed, style):
        mm, ms = mean_std(m, eps)
        sm, ss = mean_std(s, eps)
        t = F.mse_loss(mm.float(), sm.float()) + F.mse_loss(ms.float(), ss.float())
        total = t if total is None else total + t
    if total is None:
        raise ValueError("style_stats_loss: no feature pairs")
    return total


def mean_std(x: Tensor, eps: float = 1e-5) -> Tuple[Tensor, Tensor]:
    """Per-(n, c) spatial mean and ``sqrt(unbiased var + eps)`` as f32 ``[N, C]`` tensors."""
    if use_native(x) and x.dtype in _FLOATS and _layout_ok(x) and x.numel() > 0:
        return _MeanStdFn.apply(x, float(eps))
    return mean_std_ref(x, eps)
