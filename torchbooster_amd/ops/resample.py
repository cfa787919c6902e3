"""NHWC reflection padding and nearest-neighbour upsampling.

The StyleNet / AdaIN decoder blocks are ``ReflectionPad2d(k//2) + Conv`` and
``Upsample(x2) + ConvIN`` (/root/reference/examples/img_stt/online/online.py:46-48,
/root/reference/examples/img_stt/adain/adain.py:36-38).  Their activations are
channels_last bf16 here, where ATen's pad/upsample kernels run the NCHW index
math over strided memory; ``csrc/aux_ops.hip`` does both on the NHWC layout
with channel-fastest (coalesced) threads.  The backward passes are gathers —
each input pixel sums the output pixels that map onto it — so they are
deterministic and need no atomics.
"""
from __future__ import annotations

from typing import Sequence, Union

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor
from torch.autograd.function import once_differentiable

from torchbooster_amd.ops._ext import native, use_native

__all__ = ["reflection_pad2d", "upsample_nearest2d", "ReflectionPad2d", "UpsampleNearest2d"]


def _nhwc(x: Tensor) -> bool:
    return (x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and x.is_contiguous(memory_format=torch.channels_last) and x.numel() > 0)


class _RPadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pads):
        ctx.hw = (x.size(2), x.size(3))
        ctx.pads = pads
        return native().reflect_pad_forward(x, *pads)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        return native().reflect_pad_backward(g, ctx.hw[0], ctx.hw[1], *ctx.pads), None


class _UpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, f):
        ctx.f = f
        return native().upsample_nearest_forward(x, f)

    @staticmethod
    @once_differentiable
    def backward(ctx, g):
        return native().upsample_nearest_backward(g, ctx.f), None


def reflection_pad2d(x: Tensor, padding: Union[int, Sequence[int]]) -> Tensor:
    """``F.pad(x, (l, r, t, b), mode="reflect")``; native for channels_last GPU tensors."""
    pads = (padding,) * 4 if isinstance(padding, int) else tuple(int(p) for p in padding)
    if use_native(x) and _nhwc(x) and max(pads[0], pads[1]) < x.size(3) and max(pads[2], pads[3]) < x.size(2) \
            and min(pads) >= 0:
        return _RPadFn.apply(x, pads)
    return F.pad(x, pads, mode="reflect")


def upsample_nearest2d(x: Tensor, scale_factor: int = 2) -> Tensor:
    """Nearest-neighbour upsampling by an integer factor."""
    f = int(scale_factor)
    if use_native(x) and _nhwc(x) and f == scale_factor and f >= 1:
        return _UpFn.apply(x, f)
    return F.interpolate(x, scale_factor=scale_factor, mode="nearest")


class ReflectionPad2d(nn.ReflectionPad2d):
    def forward(self, x: Tensor) -> Tensor:
        return reflection_pad2d(x, self.padding)


class UpsampleNearest2d(nn.Upsample):
    def __init__(self, scale_factor: int = 2):
        super().__init__(scale_factor=scale_factor, mode="nearest")

    def forward(self, x: Tensor) -> Tensor:
        if isinstance(self.scale_factor, (int, float)) and float(self.scale_factor).is_integer():
            return upsample_nearest2d(x, int(self.scale_factor))
        return super().forward(x)
