"""Linear layer whose weight/bias gradients land in zero-copy gradient slots.

Forward and both backward GEMMs run on hipBLASLt (plain library GEMMs); what
this adds over ``nn.Linear`` is the backward writing ``dW = dYᵀ X`` and
``db = Σ dY`` straight into the parameter's persistent gradient slot
(ops/_ext.py ``take_slot``) — no accumulate-add or bucket copy per step.
State-dict compatible with ``nn.Linear``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops._ext import slot_alias, take_slot

__all__ = ["Linear", "linear"]


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
            s = take_slot(wp) if slots_ok else None
            if s is not None and s.dtype == dy.dtype and s.is_contiguous():
                torch.mm(dy2.t(), x2, out=s)
                dw = slot_alias(s)
            else:
                dw = dy2.t() @ x2
        if ctx.has_bias and ctx.needs_input_grad[2]:
            s = take_slot(bp) if slots_ok else None
            if s is not None and s.dtype == dy.dtype and s.is_contiguous():
                torch.sum(dy2, 0, out=s)
                db = slot_alias(s)
            else:
                db = dy2.sum(0)
        return dx, dw, db


def linear(x: Tensor, w: Tensor, b: Optional[Tensor] = None) -> Tensor:
    if x.is_cuda and torch.is_grad_enabled() and (w.requires_grad or (b is not None and b.requires_grad)):
        return _LinearFn.apply(x, w, b)
    return F.linear(x, w, b)


class Linear(nn.Linear):
    """``nn.Linear`` with slot-aware backward (see module docstring)."""

    def forward(self, x: Tensor) -> Tensor:
        return linear(x, self.weight, self.bias)
