"""Max-pooling on the native NHWC kernels (csrc/pool.hip).

``nn.MaxPool2d`` in the reference's VGG feature extractors
(/root/reference/examples/img_stt/offline/offline.py:104, online.py:166,
adain.py:179 via torchvision ``vgg.features``) and LeNet
(examples/img_cls/lenet/lenet.py:30-31).  The forward is the BN+act+pool
kernel with an identity affine: one read of the input, the pooled tensor and a
1-byte window argmax written; the backward is the argmax GATHER (every input
pixel sums the output grads whose argmax is its tap — no atomics, no 64-bit
index tensor as in ATen's NHWC max-pool).
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops._ext import native, use_native

__all__ = ["MaxPool2d", "max_pool2d"]

_AFFINE: Dict[Tuple[int, torch.device], Tuple[Tensor, Tensor]] = {}


def _identity_affine(C: int, dev: torch.device) -> Tuple[Tensor, Tensor]:
    key = (C, dev)
    if key not in _AFFINE:
        _AFFINE[key] = (torch.ones(C, device=dev), torch.zeros(C, device=dev))
    return _AFFINE[key]


def _pair(v) -> int:
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            return -1
        return int(v[0])
    return int(v)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        one, zero = _identity_affine(x.shape[1], x.device)
        y, idx = native().bn_act_maxpool(x, one, zero, 0, 0.0, k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (k, s, p, x.shape[2], x.shape[3])
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        k, s, p, H, W = ctx.cfg
        if torch.is_grad_enabled():  # create_graph: a differentiable gather
            raise RuntimeError("native max-pool backward is not twice differentiable")
        return native().maxpool_backward(dy, idx, H, W, k, s, p), None, None, None


def _native_ok(x: Tensor, k: int, s: int, p: int, dilation, ceil_mode: bool, return_indices: bool) -> bool:
    return (use_native(x) and x.dim() == 4 and x.shape[1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32,
                                                                                    torch.float16)
            and k > 0 and s > 0 and 0 <= p < k and k <= 16 and _pair(dilation) == 1 and not ceil_mode
            and not return_indices and x.is_contiguous(memory_format=torch.channels_last))


def max_pool2d(x: Tensor, kernel_size, stride=None, padding=0, dilation=1, ceil_mode: bool = False,
               return_indices: bool = False):
    k = _pair(kernel_size)
    s = _pair(stride if stride is not None else kernel_size)
    p = _pair(padding)
    if min(k, s, p + 1) > 0 and _native_ok(x, k, s, p, dilation, ceil_mode, return_indices):
        return _MaxPoolFn.apply(x, k, s, p)
    return F.max_pool2d(x, kernel_size, stride, padding, dilation, ceil_mode, return_indices)


class MaxPool2d(nn.MaxPool2d):
    """``nn.MaxPool2d`` on the native NHWC gather kernels when it applies (square
    window <= 16, C % 8 == 0, channels_last, no dilation / ceil_mode / indices)."""

    def forward(self, x: Tensor):
        return max_pool2d(x, self.kernel_size, self.stride, self.padding, self.dilation, self.ceil_mode,
                          self.return_indices)
