"""Gram matrices of NHWC feature maps on the native split-K SYRK kernel (csrc/gram.hip).

K18 of SURVEY.md §2.3.1: the style losses of the reference's img_stt examples
(/root/reference/examples/img_stt/online/online.py:60-63 per-sample ``bmm``,
/root/reference/examples/img_stt/offline/offline.py:25-28 whole-image matmul).

Forward: ``G[b] = F_bᵀ F_b · scale`` (f32 out) from the channels_last feature
map with no NCHW transpose; only the upper-triangle tiles are computed.
Backward: ``dF_b = F_b (dG_b + dG_bᵀ) · scale`` — one native pass builds the bf16
symmetric operand (``gram_sym``), then one native GEMM per sample (the NT engine
of csrc/gemm.hip / gemm8.hip: the operand is symmetric, so ``F_b S_b = F_b S_bᵀ``).
Native path: CUDA bf16 channels_last features with C % 64 == 0.  f32 features (the
reference's precision, offline.yml / online.yml ``fp16: false``) run on the exact-f32
MFMA kernels of the generic conv family (csrc/conv_any.hip): the Gram is the weight
gradient of a 1x1 conv whose output gradient is the input itself
(``G = Σ_pix F[pix]ᵀ F[pix]``), its backward a 1x1 conv of F with the symmetric
``(dG + dGᵀ)·scale`` as the weight.  Otherwise the PyTorch math below.
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
        from torchbooster_amd.ops import gemm as G

        (f,) = ctx.saved_tensors
        B, C, H, W = f.shape
        sym = native().gram_sym(dg.float(), ctx.scale)  # [B, C, C] bf16, symmetric
        rows = f.permute(0, 2, 3, 1).reshape(B, H * W, C)  # NHWC rows, a free view
        df = torch.empty(B, H * W, C, device=f.device, dtype=f.dtype)
        for b in range(B):
            G.mm_nt(rows[b], sym[b], out=df[b], blas=False)  # rows_b sym_bᵀ = rows_b sym_b
        return df.view(B, H, W, C).permute(0, 3, 1, 2), None


def native_f32_supported(f: Tensor) -> bool:
    return (f.is_cuda and f.dtype == torch.float32 and f.dim() == 4 and use_native(f)
            and f.is_contiguous(memory_format=torch.channels_last))


class _GramF32Fn(torch.autograd.Function):
    """Per-sample f32 Gram on the exact-f32 MFMA conv kernels (see module docstring)."""

    @staticmethod
    def forward(ctx, f, scale):
        ctx.save_for_backward(f)
        ctx.scale = scale
        C = native()
        gs = [C.conv_any_wgrad(f[b: b + 1], f[b: b + 1], 1, 1, 1, 0, 1, False) for b in range(f.shape[0])]
        return torch.stack([g.view(f.shape[1], f.shape[1]) for g in gs]).mul_(scale)

    @staticmethod
    @once_differentiable
    def backward(ctx, dg):
        (f,) = ctx.saved_tensors
        B, Cc = f.shape[0], f.shape[1]
        sym = (dg + dg.transpose(1, 2)) * ctx.scale  # [B, C, C] f32, symmetric
        C = native()
        df = [C.conv_any_fwd(f[b: b + 1], sym[b].reshape(Cc, Cc, 1, 1).contiguous(memory_format=torch.channels_last),
                             None, 1, 0, 1, False) for b in range(B)]
        return torch.cat(df, 0), None


def gram(features: Tensor, scale: float) -> Tensor:
    """[B, C, H, W] -> [B, C, C] f32 Gram ``F Fᵀ · scale`` (per sample)."""
    if native_supported(features):
        return _GramFn.apply(features, float(scale))
    if native_f32_supported(features):
        return _GramF32Fn.apply(features, float(scale))
    return gram_ref(features, scale)
