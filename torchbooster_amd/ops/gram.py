"""Gram matrices of NHWC feature maps on the native split-K SYRK kernel (csrc/gram.hip).

K18 of SURVEY.md §2.3.1: the style losses of the reference's img_stt examples
(/root/reference/examples/img_stt/online/online.py:60-63 per-sample ``bmm``,
/root/reference/examples/img_stt/offline/offline.py:25-28 whole-image matmul).

Forward: ``G[b] = F_bᵀ F_b · scale`` (f32 out) from the channels_last feature
map with no NCHW transpose; only the upper-triangle tiles are computed.
Backward: ``dF_b = F_b (dG_b + dG_bᵀ) · scale`` — one plain GEMM (hipBLASLt).
Native path: CUDA bf16 channels_last features with C % 64 == 0; otherwise the
PyTorch math below.
"""
from __future__ import annotations

import torch
from torch import Tensor
from torch.autograd.function import once_differentiable

from torchbooster_amd.ops._ext import native, use_native

__all__ = ["gram", "gram_ref", "native_supported"]


def gram_ref(features: Tensor, scale: float) -> Tensor:
    """[B, C, H, W] -> [B, C, C] f32, ``F Fᵀ * scale`` with F = [B, C, HW]."""
    B, C, H, W = features.shape
    f = features.reshape(B, C, H * W).float()
    return torch.bmm(f, f.transpose(1, 2)) * scale


def native_supported(f: Tensor) -> bool:
    return (f.is_cuda and f.dtype == torch.bfloat16 and f.dim() == 4 and f.shape[1] % 64 == 0
            and f.is_contiguous(memory_format=torch.channels_last) and use_native(f))


class _GramFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, f, scale):
        ctx.save_for_backward(f)
        ctx.scale = scale
        return native().gram_forward(f, scale)

    @staticmethod
    @once_differentiable
    def backward(ctx, dg):
        (f,) = ctx.saved_tensors
        B, C, H, W = f.shape
        sym = (dg + dg.transpose(1, 2)).mul_(ctx.scale).to(f.dtype)  # [B, C, C]
        rows = f.permute(0, 2, 3, 1).reshape(B, H * W, C)  # NHWC rows, a free view
        df = torch.bmm(rows, sym)  # [B, HW, C]
        return df.view(B, H, W, C).permute(0, 3, 1, 2), None


def gram(features: Tensor, scale: float) -> Tensor:
    """[B, C, H, W] -> [B, C, C] f32 Gram ``F Fᵀ · scale`` (per sample)."""
    if native_supported(features):
        return _GramFn.apply(features, float(scale))
    return gram_ref(features, scale)
