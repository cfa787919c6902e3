"""Linear layers on the native GEMM engine (csrc/gemm.hip, ops/gemm.py).

Reference: ``nn.Linear`` in every example MLP / head
(/root/reference/examples/img_gen/gan/gan.py:35-48, vae.py:37-55,
img_cls/lenet/lenet.py:33-35, resnet.py:112) -> cuBLAS.  Here, per step:

* forward  ``y = x Wᵀ + b`` (bias fused; ``LinearGELU`` also fuses the exact
  GELU and saves the pre-activation for its backward);
* input gradient ``dX = dY W`` (W read transposed from LDS, no Wᵀ copy);
* weight gradient ``dW = dYᵀ X`` (split-K over the batch x tokens rows);
* ``db = Σ dY`` — a native column sum (``LinearGELU``: fused with GELU').

Weight/bias gradients land straight in the parameter's persistent gradient
slot (ops/_ext.py ``take_slot``) — no accumulate-add or bucket copy per step.
Shapes the engine does not take (a feature count not a multiple of 8, fp32 /
fp16 activations) use ATen.  State-dict compatible with ``nn.Linear``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops import gemm as G
from torchbooster_amd.ops._ext import native, slot_alias, take_slot, use_native

__all__ = ["Linear", "linear", "LinearGELU", "linear_gelu", "GeluLink"]

# The fused epilogue stages the z tile through LDS with coalesced 16-B loads: 0.221 vs 0.273 ms
# unfused, ViT-B/16 5245 / 5241 vs 5134 / 5137 img/s alternated (profiles/r03_gemm_nn/README.md;
# its first form, 8-B z loads in the accumulator layout, lost in the real step on a cold z).
# TBAMD_FUSE_GELU_BWD=0 turns it off.
_FUSE_GELU_BWD = os.environ.get("TBAMD_FUSE_GELU_BWD", "1") == "1"


class GeluLink:
    """``LinearGELU`` (fc1) -> ``Linear`` (fc2) hand-off of the MLP backward.

    fc2's input gradient dH = dY W2 is only ever multiplied by GELU'(z1) (fc1's backward), and
    fc1's bias gradient is the column sum of that product: with a link, fc2's backward computes
    dZ1 = (dY W2) * GELU'(z1) and Σ dZ1 in ONE GEMM epilogue (csrc/gemm8.hip NN mode,
    ``gemm_nn_gelu_bwd``) and hands dZ1 to autograd as "the gradient of H"; fc1's backward
    recognises that very tensor and skips its own GELU / bias pass.  Only valid when fc2 is
    H's sole consumer (the caller wires it that way, e.g. models/vit.py MLP)."""

    __slots__ = ("z", "bias", "dz_ptr", "db")

    def __init__(self) -> None:
        self.z = self.bias = self.dz_ptr = self.db = None

    def take(self, dy: Tensor):
        """(True, bias gradient) when ``dy`` is the fused dZ this link handed out, else (False, None)."""
        ptr, db = self.dz_ptr, self.db
        self.dz_ptr = self.db = None
        if ptr is None:
            return False, None
        if ptr == dy.data_ptr():
            return True, db
        # fc2 already applied GELU' to what it handed out: a different tensor here means a
        # tensor hook or a second consumer rewrote H's gradient, and recomputing GELU' on it
        # would apply it twice -- fail closed instead of returning a wrong gradient
        raise RuntimeError("GeluLink: the hidden activation's gradient was modified between fc2 and fc1 "
                           "(tensor hook or second consumer); build the MLP without gelu_in for this use")


def _wgrad(dy2: Tensor, x2: Tensor, wp: Tensor) -> Tensor:
    """dW = dy2ᵀ x2 into ``wp``'s gradient slot when it has one."""
    s = take_slot(wp)
    if s is not None and not (s.dtype == dy2.dtype and s.is_contiguous()):
        s = None
    if G.supported_tn(dy2, x2):
        dw = G.mm_tn(dy2, x2, out=s)
        return slot_alias(s) if s is not None else dw

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


# the fused GELU-backward product on the cached transposed weight (row-read NT kernel) instead of the
# NN kernel's transposing reads (ops/conv.py transposed_linear_weight); TBAMD_GELU_BWD_NT=0: NN (A/B)
_GELU_BWD_NT = os.environ.get("TBAMD_GELU_BWD_NT", "1") == "1"


def _gelu_fused_dx(dy2: Tensor, w: Tensor, link: Optional[GeluLink], x_shape,
                   owner: Optional[Tensor] = None) -> Optional[Tensor]:
    """fc2's input gradient fused with fc1's GELU backward + bias gradient (GeluLink)."""
    if link is None or link.z is None or not _FUSE_GELU_BWD:
        return None
    z2 = link.z.reshape(-1, link.z.shape[-1])
    K, Q = w.shape
    if not (dy2.dtype == w.dtype == z2.dtype == torch.bfloat16 and dy2.is_cuda and K % 64 == 0 and Q % 8 == 0
            and tuple(z2.shape) == (dy2.shape[0], Q) and dy2.stride(-1) == 1 and dy2.stride(0) % 8 == 0):
        return None
    bp = link.bias
    sb = take_slot(bp) if bp is not None else None
    if sb is not None and not (sb.dtype == torch.bfloat16 and sb.is_contiguous()):
        sb = None
    wt = None
    if _GELU_BWD_NT and owner is not None:
        from torchbooster_amd.ops.conv import transposed_linear_weight

        wt = transposed_linear_weight(w, owner)
    dz, db = native().gemm_nn_gelu_bwd(dy2, w, z2, sb, wt)
    link.dz_ptr = dz.data_ptr()
    link.db = slot_alias(sb) if sb is not None else db.to(bp.dtype) if bp is not None else None
    return dz.view(*x_shape[:-1], Q)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gelu_in=None):
        ctx.save_for_backward(x, w)
        ctx.params = (w, b)
        ctx.has_bias = b is not None
        ctx.gelu_in = gelu_in
        return _fwd(x, w, b)

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
            dx = _gelu_fused_dx(dy2, w, ctx.gelu_in, x.shape, wp) if slots_ok else None
            if dx is None:
                dx = G.mm_nn(dy, w, owner=wp) if (slots_ok and G.supported_nn(dy, w)) else dy @ w
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
        return dx, dw, db, None


def _fwd(x: Tensor, w: Tensor, b: Optional[Tensor]) -> Tensor:
    if G.supported_nt(x, w) and (b is None or b.dtype == torch.bfloat16):
        return G.mm_nt(x, w, b)
    return F.linear(x, w, b)


def linear(x: Tensor, w: Tensor, b: Optional[Tensor] = None, gelu_in: Optional[GeluLink] = None) -> Tensor:
    """``gelu_in``: ``x`` is the output of the ``LinearGELU`` holding this link (its sole consumer)."""
    if use_native(x) and not torch.is_autocast_enabled("cuda"):
        if torch.is_grad_enabled() and (w.requires_grad or (b is not None and b.requires_grad)
                                        or x.requires_grad):
            return _LinearFn.apply(x, w, b, gelu_in)
        return _fwd(x, w, b)
    return F.linear(x, w, b)


class Linear(nn.Linear):
    """``nn.Linear`` with slot-aware backward (see module docstring)."""

    def forward(self, x: Tensor, act: Optional[str] = None, gelu_in: Optional[GeluLink] = None) -> Tensor:
        """``act="gelu"``: exact GELU fused into this call (nativize's Linear -> GELU fusion);
        ``gelu_in``: see :class:`GeluLink`."""
        if act == "gelu":
            return linear_gelu(x, self.weight, self.bias)
        if act not in (None, "none", "identity"):
            raise ValueError(f"Linear: unsupported fused activation {act!r}")
        return linear(x, self.weight, self.bias, gelu_in)


class _LinearGELUFn(torch.autograd.Function):
    """y = GELU(x Wᵀ + b).  Forward: one native GEMM whose epilogue adds the
    bias, applies the exact GELU and also stores z (saved for backward).
    Backward: ONE native pass computes dZ = dY·GELU'(z) and the bias gradient
    Σ dZ together (csrc/colsum.hip), then the two native GEMMs."""

    @staticmethod
    def forward(ctx, x, w, b, link=None):
        if G.supported_nt(x, w) and b is not None and b.dtype == torch.bfloat16:
            y, z = G.mm_nt(x, w, b, gelu=True)  # bias + GELU in the GEMM epilogue, z saved
        else:
            z = F.linear(x, w, b)
            y = F.gelu(z)
        ctx.save_for_backward(x, w, z)
        ctx.params = (w, b)
        ctx.link = link
        if link is not None:
            link.z, link.bias, link.dz_ptr, link.db = z, b, None, None
        return y

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
            return dx, dw, db, None
        C = dy.shape[-1]
        fused, link_db = ctx.link.take(dy) if ctx.link is not None else (False, None)
        if ctx.link is not None:
            ctx.link.z = None
        if fused:
            # fc2's backward already applied GELU' and summed the bias gradient (GeluLink)
            dz, db = dy.reshape(-1, C), link_db
        else:
            dy2, z2 = dy.reshape(-1, C), z.reshape(-1, C)
            sb = take_slot(bp) if bp is not None else None
            if sb is not None and not (sb.dtype == z.dtype and sb.is_contiguous()):
                sb = None
            dz, db = native().gelu_bwd_colsum(dy2, z2, sb)
            if sb is not None:
                db = slot_alias(sb)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = (G.mm_nn(dz, w, owner=wp) if G.supported_nn(dz, w) else dz @ w).view(*x.shape[:-1], w.shape[1])
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dz, x.reshape(-1, x.shape[-1]), wp)
        return dx, dw, (db if bp is not None and ctx.needs_input_grad[2] else None), None


def linear_gelu(x: Tensor, w: Tensor, b: Optional[Tensor] = None, link: Optional[GeluLink] = None) -> Tensor:
    """GELU(linear(x)) with the fused native backward on GPU (``link``: see :class:`GeluLink`)."""
    if use_native(x) and not torch.is_autocast_enabled("cuda") and w.shape[0] % 8 == 0:
        if torch.is_grad_enabled() and (w.requires_grad or (b is not None and b.requires_grad) or x.requires_grad):
            return _LinearGELUFn.apply(x, w, b, link)
        if G.supported_nt(x, w) and b is not None and b.dtype == torch.bfloat16:
            return G.mm_nt(x, w, b, gelu=True)[0]
    return F.gelu(F.linear(x, w, b))


class LinearGELU(nn.Linear):
    """``nn.Linear`` followed by exact GELU (state-dict compatible with ``nn.Linear``)."""

    def forward(self, x: Tensor, link: Optional[GeluLink] = None) -> Tensor:
        return linear_gelu(x, self.weight, self.bias, link)
