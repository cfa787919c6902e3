"""Fused multi-head attention on the native flash-style MFMA kernels (csrc/attention.hip).

Not in the reference (no attention model): K26 of SURVEY.md
§2.3.1, for the ViT-B/16 north-star configuration.

* :func:`attention_packed` takes the packed ``[B, N, 3*H*D]`` output of a QKV
  projection and returns ``[B, N, H*D]`` — the layout the output projection
  reads — with no permute/contiguous copies in either direction: the kernels
  read q/k/v through strides and the backward writes dq/dk/dv straight into one
  packed ``dqkv`` buffer.
* :func:`attention` takes ``[B, H, N, D]`` q, k, v (any strides).

Native path: CUDA bf16 tensors with head dim 64.  Everything else (CPU, other
dtypes/head dims, ``TBAMD_FORCE_REFERENCE=1`` comparator runs) takes stock
``F.scaled_dot_product_attention``; :func:`attention_ref` is the explicit fp32
math the GPU tests compare against.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor
from torch.autograd.function import once_differentiable

from torchbooster_amd.ops._ext import native, use_native

__all__ = ["attention", "attention_packed", "attention_ref", "native_supported"]


def attention_ref(q: Tensor, k: Tensor, v: Tensor, scale: Optional[float] = None) -> Tensor:
    """softmax(q kᵀ · scale) v over [..., N, D] tensors (f32 softmax)."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    s = torch.matmul(q, k.transpose(-1, -2)) * scale
    p = torch.softmax(s.float(), dim=-1).to(q.dtype)
    return torch.matmul(p, v)


def native_supported(q: Tensor) -> bool:
    return q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] == 64 and use_native(q)


class _AttnFn(torch.autograd.Function):
    """q, k, v: [B, H, N, 64] views -> o [B, N, H, 64] (contiguous)."""

    @staticmethod
    def forward(ctx, q, k, v, scale):
        o, lse = native().attn_forward(q, k, v, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.scale = scale
        return o

    @staticmethod
    @once_differentiable
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = do.contiguous()
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        native().attn_backward(q, k, v, o.permute(0, 2, 1, 3), do.permute(0, 2, 1, 3), lse, ctx.scale, dq, dk, dv)
        return dq, dk, dv, None


class _AttnPackedFn(torch.autograd.Function):
    """qkv: [B, N, 3*H*64] -> [B, N, H*64]; the gradient is one packed buffer."""

    @staticmethod
    def forward(ctx, qkv, heads, scale):
        B, N, E3 = qkv.shape
        D = E3 // (3 * heads)
        t = qkv.view(B, N, 3, heads, D)
        q, k, v = (t[:, :, i].transpose(1, 2) for i in range(3))
        o, lse = native().attn_forward(q, k, v, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.cfg = (heads, D, scale)
        return o.view(B, N, heads * D)

    @staticmethod
    @once_differentiable
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        heads, D, scale = ctx.cfg
        B, N, _ = qkv.shape
        t = qkv.view(B, N, 3, heads, D)
        dqkv = torch.empty_like(qkv)
        g = dqkv.view(B, N, 3, heads, D)
        do = do.contiguous().view(B, N, heads, D)
        native().attn_backward(t[:, :, 0].transpose(1, 2), t[:, :, 1].transpose(1, 2), t[:, :, 2].transpose(1, 2),
                               o.permute(0, 2, 1, 3), do.permute(0, 2, 1, 3), lse, scale,
                               g[:, :, 0].transpose(1, 2), g[:, :, 1].transpose(1, 2), g[:, :, 2].transpose(1, 2))
        return dqkv, None, None


def _rows_ok(t: Tensor) -> bool:
    return t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:-1]) and t.data_ptr() % 16 == 0


def attention(q: Tensor, k: Tensor, v: Tensor, scale: Optional[float] = None) -> Tensor:
    """[B, H, N, D] -> [B, H, N, D]."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else float(scale)
    if native_supported(q) and q.dim() == 4 and q.shape == k.shape == v.shape:
        q, k, v = (x if _rows_ok(x) else x.contiguous() for x in (q, k, v))
        return _AttnFn.apply(q, k, v, scale).permute(0, 2, 1, 3)
    # stock PyTorch (the comparator of --mode stock benchmarks; CPU path)
    return F.scaled_dot_product_attention(q, k, v, scale=scale)


def attention_packed(qkv: Tensor, heads: int, scale: Optional[float] = None) -> Tensor:
    """[B, N, 3*H*D] packed q|k|v (head-major inside each) -> [B, N, H*D]."""
    B, N, E3 = qkv.shape
    D = E3 // (3 * heads)
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    if native_supported(qkv.view(B, N, 3, heads, D)) and _rows_ok(qkv):
        return _AttnPackedFn.apply(qkv, heads, scale)
    t = qkv.view(B, N, 3, heads, D).permute(2, 0, 3, 1, 4)
    o = F.scaled_dot_product_attention(t[0], t[1], t[2], scale=scale)
    return o.transpose(1, 2).reshape(B, N, heads * D)
