"""NHWC convolution on the native implicit-GEMM MFMA kernel (csrc/conv.hip).

``conv2d(x, w, bias, stride, padding)`` runs the HIP kernel when the shape is
supported (bf16, groups=1, dilation=1, square stride/padding, C_in % 64 == 0,
C_out % 64 == 0) and falls back to ATen (MIOpen) otherwise.  Backward:

* input grad of a stride-1 conv = the same forward kernel on dY with the
  flipped, transposed weights (``conv_flip_weight``) and padding R-1-pad;
* other input grads and the weight grad go through ATen's
  ``convolution_backward`` (MIOpen) for now.

:func:`conv2d_bn_stats` additionally returns per-tile BatchNorm partial sums
emitted by the conv epilogue (used by :class:`~torchbooster_amd.models.resnet.ConvBNAct`).
Reference: every Conv2d of the examples.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from torchbooster_amd.ops._ext import native, use_native

__all__ = ["conv2d", "conv2d_bn_stats", "native_supported", "conv2d_forward"]

_DISABLE = os.environ.get("TBAMD_NATIVE_CONV", "1") == "0"


def _pair(v) -> int:
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            return -1
        return int(v[0])
    return int(v)


def native_supported(x: Tensor, w: Tensor, stride, padding, dilation=1, groups=1) -> bool:
    if _DISABLE or not x.is_cuda or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if groups != 1 or _pair(dilation) != 1 or _pair(stride) < 1 or _pair(padding) < 0:
        return False
    if w.shape[2] != w.shape[3]:
        return False
    C, K = x.shape[1], w.shape[0]
    return C % 64 == 0 and K % 64 == 0


def conv2d_forward(x: Tensor, w: Tensor, stride: int, pad: int, bias: Optional[Tensor] = None,
                   relu: bool = False) -> Tensor:
    """Raw forward on the native kernel (no autograd)."""
    return native().conv2d_fwd(x, w, bias, stride, pad, relu, False)[0]


def _dgrad(dy: Tensor, x_shape, w: Tensor, stride: int, pad: int, x_like: Tensor) -> Tensor:
    K, C, R, S = w.shape
    if stride == 1 and K % 64 == 0 and C % 64 == 0 and pad <= R - 1:
        wt = native().conv_flip_weight(w)
        return native().conv2d_fwd(dy, wt, None, 1, R - 1 - pad, False, False)[0]
    return torch.ops.aten.convolution_backward(dy, x_like, w, None, [stride, stride], [pad, pad], [1, 1], False,
                                               [0, 0], 1, [True, False, False])[0]


def _wgrad(dy: Tensor, x: Tensor, w: Tensor, stride: int, pad: int) -> Tensor:
    return torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0],
                                               1, [False, True, False])[1]


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, want_stats):
        y, stats = native().conv2d_fwd(x, w, bias, stride, pad, False, want_stats)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, bias is not None)
        if stats is not None and stats.numel() > 0:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, dstats):
        x, w = ctx.saved_tensors
        stride, pad, has_bias = ctx.cfg
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _dgrad(dy, x.shape, w, stride, pad, x)
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dy, x, w, stride, pad)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum(dim=(0, 2, 3)).to(w.dtype)
        return dx, dw, db, None, None, None


def conv2d(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, stride=1, padding=0, dilation=1,
           groups=1) -> Tensor:
    if use_native(x) and native_supported(x, w, stride, padding, dilation, groups):
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
        return _ConvFn.apply(x, w, bias, _pair(stride), _pair(padding), False)[0]
    return F.conv2d(x, w, bias, stride, padding, dilation, groups)


def conv2d_bn_stats(x: Tensor, w: Tensor, stride: int, padding: int) -> Tuple[Tensor, Optional[Tensor]]:
    """Native conv returning (y, bn_partials) or (ATen conv, None) when unsupported."""
    if use_native(x) and native_supported(x, w, stride, padding):
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
        y, stats = _ConvFn.apply(x, w, None, _pair(stride), _pair(padding), True)
        return y, stats
    return F.conv2d(x, w, None, stride, padding), None


class Conv2d(torch.nn.Conv2d):
    """``nn.Conv2d`` that runs the native implicit-GEMM kernel when it can
    (bf16 NHWC, C_in and C_out multiples of 64, groups 1, no dilation, zero
    padding) and MIOpen otherwise.  State-dict compatible with ``nn.Conv2d``."""

    def forward(self, x: Tensor) -> Tensor:
        if self.padding_mode == "zeros" and x.is_cuda and native_supported(x, self.weight, self.stride, self.padding,
                                                                          self.dilation, self.groups):
            return conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups)
        return super().forward(x)
