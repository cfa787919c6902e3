"""Linear layer whose weight/bias gradients land in zero-copy gradient slots.

Forward and input-gradient GEMMs run on hipBLASLt (plain library GEMMs).  The
weight gradient ``dW = dYᵀ X`` reduces over all M = batch x tokens rows into a
small [out, in] tile grid (768 x 768 is 36 tiles of 128² for 256 CUs), the
shape library GEMMs handle worst; it is autotuned per shape between hipBLASLt
and the native split-K MFMA weight-gradient kernel (csrc/conv_wgrad.hip, the
same GEMM as a 1x1-conv wgrad over M "pixels").  ``db = Σ dY`` is a native
column sum.  Both land straight in the parameter's persistent gradient slot
(ops/_ext.py ``take_slot``) — no accumulate-add or bucket copy per step.
State-dict compatible with ``nn.Linear``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops._ext import native, slot_alias, take_slot, use_native

__all__ = ["Linear", "linear", "LinearGELU", "linear_gelu"]


def _wgrad(dy2: Tensor, x2: Tensor, wp: Tensor) -> Tensor:
    """dW = dy2ᵀ x2 into ``wp``'s gradient slot when it has one (autotuned route)."""
    s = take_slot(wp)
    if s is not None and not (s.dtype == dy2.dtype and s.is_contiguous()):
        s = None

    def blas():
        if s is not None:
            torch.mm(dy2.t(), x2, out=s)
            return slot_alias(s)
        return dy2.t() @ x2

    M, K = dy2.shape
    C = x2.shape[1]
    if not (dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and K % 64 == 0 and C % 64 == 0
            and M >= 4096 and dy2.is_cuda):
        return blas()

    def nat():
        dy4, x4 = dy2.contiguous().view(M, K, 1, 1), x2.contiguous().view(M, C, 1, 1)
        if s is not None:
            native().conv2d_wgrad(dy4, x4, 1, 1, 1, 0, s.view(K, C, 1, 1))
            return slot_alias(s)
        return native().conv2d_wgrad(dy4, x4, 1, 1, 1, 0).view(K, C)

    from torchbooster_amd.ops.conv import _route

    return _route("wgrad", ("linear", M, K, C), [("hipblaslt", blas, 0.0), ("native", nat, 0.0)])


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.params = (w, b)
        ctx.has_bias = b is not None
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        wp, bp = ctx.params
        dx = dw = db = None
        dy2 = dy.reshape(-1, dy.shape[-1])
        # under create_graph (double backward, e.g. a GAN gradient penalty) the
        # ops below are recorded: no out= writes into gradient slots then
        slots_ok = not torch.is_grad_enabled()
        if ctx.needs_input_grad[0]:
            dx = dy @ w
        if ctx.needs_input_grad[1]:
            x2 = x.reshape(-1, x.shape[-1])
            dw = _wgrad(dy2, x2, wp) if slots_ok else dy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            s = take_slot(bp) if slots_ok else None
            if s is not None and not (s.dtype == dy.dtype and s.is_contiguous()):
                s = None
            if slots_ok and dy2.shape[-1] % 8 == 0:
                db = native().colsum(dy2, s)  # native column sum (into the slot when there is one)
                if s is not None:
                    db = slot_alias(s)
            elif s is not None:
                torch.sum(dy2, 0, out=s)
                db = slot_alias(s)
            else:
                db = dy2.sum(0)
        return dx, dw, db


def linear(x: Tensor, w: Tensor, b: Optional[Tensor] = None) -> Tensor:
    if (use_native(x) and torch.is_grad_enabled() and not torch.is_autocast_enabled("cuda")
            and (w.requires_grad or (b is not None and b.requires_grad))):
        return _LinearFn.apply(x, w, b)
    return F.linear(x, w, b)


class Linear(nn.Linear):
    """``nn.Linear`` with slot-aware backward (see module docstring)."""

    def forward(self, x: Tensor) -> Tensor:
        return linear(x, self.weight, self.bias)


class _LinearGELUFn(torch.autograd.Function):
    """y = GELU(x Wᵀ + b).  Forward: one hipBLASLt GEMM with the bias epilogue +
    the GELU pass (z is saved).  Backward: ONE native pass computes
    dZ = dY·GELU'(z) and the bias gradient Σ dZ together (csrc/colsum.hip),
    then the two weight/input GEMMs."""

    @staticmethod
    def forward(ctx, x, w, b):
        z = F.linear(x, w, b)
        ctx.save_for_backward(x, w, z)
        ctx.params = (w, b)
        return F.gelu(z)

    @staticmethod
    def backward(ctx, dy):
        x, w, z = ctx.saved_tensors
        wp, bp = ctx.params
        if torch.is_grad_enabled():  # create_graph (double backward): differentiable math on the saved inputs
            zz = F.linear(x, w, bp)
            gp = 0.5 * (1.0 + torch.erf(zz * 0.7071067811865476)) + zz * torch.exp(-0.5 * zz * zz) * 0.3989422804014327
            dz = dy * gp
            dz2 = dz.reshape(-1, dz.shape[-1])
            dx = dz @ w
            dw = dz2.t() @ x.reshape(-1, x.shape[-1])
            db = dz2.sum(0) if bp is not None else None
            return dx, dw, db
        C = dy.shape[-1]
        dy2, z2 = dy.reshape(-1, C), z.reshape(-1, C)
        sb = take_slot(bp) if bp is not None else None
        if sb is not None and not (sb.dtype == z.dtype and sb.is_contiguous()):
            sb = None
        dz, db = native().gelu_bwd_colsum(dy2, z2, sb)
        if sb is not None:
            db = slot_alias(sb)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = (dz @ w).view(*x.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dz, x.reshape(-1, x.shape[-1]), wp)
        return dx, dw, (db if bp is not None and ctx.needs_input_grad[2] else None)


def linear_gelu(x: Tensor, w: Tensor, b: Optional[Tensor] = None) -> Tensor:
    """GELU(linear(x)) with the fused native backward on GPU."""
    if (use_native(x) and torch.is_grad_enabled() and not torch.is_autocast_enabled("cuda")
            and w.shape[0] % 8 == 0 and (w.requires_grad or (b is not None and b.requires_grad))):
        return _LinearGELUFn.apply(x, w, b)
    return F.gelu(F.linear(x, w, b))


class LinearGELU(nn.Linear):
    """``nn.Linear`` followed by exact GELU (state-dict compatible with ``nn.Linear``)."""

    def forward(self, x: Tensor) -> Tensor:
        return linear_gelu(x, self.weight, self.bias)
