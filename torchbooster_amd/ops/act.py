"""Standalone activations on the native elementwise kernels (csrc/aux_ops.hip ``act_fwd_k`` /
``act_bwd_k``): the activations nothing upstream can absorb -- e.g. the LeakyReLU(0.2) after the
DCGAN discriminator's bias-only input conv, or a stock ``nn.LeakyReLU`` / ``nn.GELU`` that
:func:`~torchbooster_amd.nativize` finds after an op without an activation epilogue.  The
backward recomputes act'(x) from the saved input (the reference: ATen's ``leaky_relu`` /
``leaky_relu_backward`` kernels behind ``nn.LeakyReLU``, examples/img_gen/gan/gan.py:37-46).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops._ext import native, use_native
from torchbooster_amd.ops.norm import ACT_CODES, act_ref

__all__ = ["activation", "leaky_relu", "LeakyReLU"]


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, code, slope):
        ctx.save_for_backward(x)
        ctx.cfg = (code, slope)
        return native().act_fwd(x, code, slope)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        code, slope = ctx.cfg
        if torch.is_grad_enabled():  # double backward: differentiable recompute
            name = {v: k for k, v in ACT_CODES.items() if isinstance(k, str)}[code]
            with torch.enable_grad():
                xx = x.detach().requires_grad_(True)
                y = act_ref(xx, name, slope)
                (g,) = torch.autograd.grad(y, xx, dy, create_graph=True)
            return g, None, None
        return native().act_bwd(x, dy.to(x.dtype), code, slope), None, None


def activation(x: Tensor, act: str, slope: float = 0.01) -> Tensor:
    """``act`` in {"relu", "gelu", "silu", "leaky_relu"} on the native kernels (GPU, numel % 8 == 0)."""
    code = ACT_CODES[act]
    if use_native(x) and x.is_floating_point() and x.numel() % 8 == 0 and x.numel() > 0:
        return _ActFn.apply(x, code, float(slope))
    return act_ref(x, act, slope)


def leaky_relu(x: Tensor, negative_slope: float = 0.01) -> Tensor:
    return activation(x, "leaky_relu", negative_slope)


class LeakyReLU(nn.LeakyReLU):
    """``nn.LeakyReLU`` on the native kernels (``inplace`` is accepted and returns a new tensor)."""

    def forward(self, x: Tensor) -> Tensor:
        if use_native(x):
            return leaky_relu(x, self.negative_slope)
        return F.leaky_relu(x, self.negative_slope, self.inplace)
