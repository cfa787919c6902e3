"""Fused normalisation + activation ops.

:class:`BatchNormAct2d` is a drop-in ``BatchNorm2d`` whose forward computes
``act(bn(x) + residual)`` in one NHWC pass (HIP kernels in
``csrc/norm_bn.hip``).  Reference counterparts: ``torch.nn.BatchNorm2d`` +
``ReLU``/``GELU`` as used by the img_cls examples
(/root/reference/examples/img_cls/lenet/lenet.py:30-31, torchvision ResNet in
/root/reference/examples/img_cls/resnet/resnet.py:111).  SURVEY.md §2.3.1 K4/K5.
"""
from __future__ import annotations

import os
import weakref
from typing import Optional

import torch
from torch.autograd.function import once_differentiable
import torch.nn.functional as F
from torch import Tensor, nn

from torchbooster_amd.ops import streams
from torchbooster_amd.ops._ext import slot_alias, take_slot, native, use_native

ACT_CODES = {"none": 0, "identity": 0, None: 0, "relu": 1, "gelu": 2, "silu": 3, "leaky_relu": 4}


def act_ref(z: Tensor, act: str, slope: float = 0.01) -> Tensor:
    if act in ("none", "identity", None):
        return z
    if act == "relu":
        return F.relu(z)
    if act == "gelu":
        return F.gelu(z)
    if act == "silu":
        return F.silu(z)
    if act == "leaky_relu":
        return F.leaky_relu(z, slope)
    raise ValueError(f"unknown activation {act}")


def _to_rows(x: Tensor):
    """View an (N, C, *spatial) tensor as channels-innermost rows [M, C].

    Returns (rows, restore) where restore(rows2) maps a [M, C] result back to the
    logical shape of x (channels_last strides for 4-D input).
    """
    if x.dim() == 2:
        return x.contiguous(), lambda r: r
    N, C = x.shape[0], x.shape[1]
    if x.dim() == 4:
        xc = x.contiguous(memory_format=torch.channels_last)
        H, W = x.shape[2], x.shape[3]
        rows = xc.permute(0, 2, 3, 1).reshape(N * H * W, C)
        return rows, lambda r: r.view(N, H, W, C).permute(0, 3, 1, 2)
    spatial = x.shape[2:]
    perm = [0] + list(range(2, x.dim())) + [1]
    rows = x.permute(*perm).contiguous().reshape(-1, C)
    inv = [0, x.dim() - 1] + list(range(1, x.dim() - 1))
    return rows, lambda r: r.view(N, *spatial, C).permute(*inv)


class ResidualGradLink:
    """Hands the gradient of a ReLU-after-residual-add to the op that produced
    the residual WITHOUT materialising it.

    The BN whose forward added the residual saves a 1-bit ReLU mask instead of
    reading its output back; its backward deposits ``(dy, mask)`` here and
    returns no gradient for the residual input; the conv that handed its input
    out as that residual (``conv2d_bn_stats(..., passthrough=True, link=...)``)
    picks the pair up and adds ``dy * mask`` inside its dgrad epilogue.  The
    conv's backward always runs after the BN's (it depends on it through the
    main branch), so the hand-off is ordered by autograd itself."""

    __slots__ = ("dy", "mask", "carrier", "ver", "ds_x", "ds_mean", "ds_part")

    def __init__(self, carrier: bool = False) -> None:
        """``carrier``: the residual's producer is a BatchNorm without activation (a bottleneck's
        downsample branch) rather than a conv.  Autograd must still reach that branch, so the
        block-output BN returns the UNMASKED dy as the residual's gradient (no extra pass) and the
        downsample BN applies the mask in its own backward kernels (csrc/norm_bn.hip MASKIN): the
        masked residual gradient is never written."""
        self.dy: Optional[Tensor] = None
        self.mask: Optional[Tensor] = None
        self.carrier = carrier
        self.ver = None
        # carrier: the downsample BN's input rows / batch mean (set by its forward), and its backward
        # partial sums, which the block-output BN's backward apply accumulates on the way
        self.ds_x = self.ds_mean = self.ds_part = None

    def put(self, dy: Tensor, mask: Tensor) -> None:
        self.dy, self.mask, self.ver = dy, mask, dy._version

    def take(self):
        out = (self.dy, self.mask)
        self.dy = self.mask = self.ver = None
        return out

    def take_carried(self, g: Tensor):
        """(mask, partials or None) for the carrier gradient ``g`` the downsample BN received.  ``g``
        must be the very dy this link handed out, unmodified: anything else (a tensor hook, a second
        consumer of the residual) would need the mask applied to a different tensor -- fail closed."""
        dy, mask, ver, part = self.dy, self.mask, self.ver, self.ds_part
        self.dy = self.mask = self.ver = self.ds_part = self.ds_x = self.ds_mean = None
        if dy is None or mask is None or g.data_ptr() != dy.data_ptr() or g._version != ver or g.shape != dy.shape:
            raise RuntimeError("ResidualGradLink(carrier): the downsample branch received a gradient other than "
                               "the block output's dy (tensor hook or second consumer); build the block without "
                               "the carrier link for this use")
        return mask, part


class BnBwdLink:
    """Lets the conv that consumes a BatchNorm's output compute that BN's
    backward partial sums inside its dgrad epilogue (csrc/conv.hip BNB).

    The BN forward fills the BN input / statistics / ReLU-mask fields; the
    consumer conv's backward reads them, emits ``part`` = per-pixel-tile
    (sum dz, sum dz*(x-mean)) while writing dX, and records dX's storage;
    the BN backward — which autograd runs next, on that very dX — finalises
    from ``part`` instead of re-reading (dX, x).  Only valid when the conv's dX
    is the BN output's whole gradient (the caller wires it that way); the BN
    backward checks it received the recorded tensor and otherwise falls back."""

    __slots__ = ("xb", "mean", "scale", "shift", "bits", "mode", "part", "dx_ptr")

    def __init__(self) -> None:
        self.mode = 0
        self.xb = self.mean = self.scale = self.shift = self.bits = self.part = None
        self.dx_ptr = None

    def ready(self) -> bool:
        return self.mode != 0 and self.xb is not None

    def take(self, dy: Tensor):
        part, ptr = self.part, self.dx_ptr
        self.part = self.dx_ptr = None
        if part is None or ptr != dy.data_ptr():
            return None
        return part


class BnGradXf:
    """The BN backward apply deferred into the producing conv's input gradient (csrc/conv.hip GXF).

    A BatchNorm whose backward partial sums came from its consumer's dgrad epilogue (BnBwdLink)
    still had to write dX = ka * act'(z) * g + c0 + c1 * x (the "apply": read g and x, write dX),
    which the conv that produced x then read twice (its dgrad and its weight gradient).  With this
    link the BN backward runs only the finalize (coefficients, dgamma, dbeta), deposits
    (g, x, mask source, coefficients) here and returns a stride-0 placeholder; that conv's backward
    -- a 1x1 stride-1 conv, whose input gradient is the very next kernel -- applies the transform to
    its dgrad operand as it lands in LDS and stores the transformed tile once for its weight
    gradient.  The apply pass disappears ("reverse XF": consumer-side BN
    backward).  OPT-IN (``TBAMD_BN_GXF=1``): measured SLOWER on the ResNet-50 step, 22.68 vs 21.06
    ms under the kernel trace -- the single-stage dgrads that take the second operand stream and
    the transform cost more (conv1 dgrads 2.56 vs 1.86 ms, conv3 dgrads +1.4 ms) than the apply
    passes they remove (1.8 ms); profiles/r06_gxf/.  ``mode``: 1 = ReLU mask recomputed from
    (x, scale, shift), 2 = ReLU-after-residual mask from the saved bits.  Fail-safe: a consumer
    that cannot take it (or any other tensor arriving as its gradient) calls :meth:`materialize`."""

    __slots__ = ("g", "xb", "bits", "scale", "shift", "coef", "mode", "ph", "restore", "__weakref__")

    def __init__(self) -> None:
        self.g = self.xb = self.bits = self.scale = self.shift = self.coef = self.ph = self.restore = None
        self.mode = 0

    def ready(self, dy: Optional[Tensor]) -> bool:
        return (self.mode != 0 and dy is not None and self.ph is not None and dy.data_ptr() == self.ph.data_ptr()
                and dy.shape == self.ph.shape and dy.stride() == self.ph.stride())

    def take(self):
        out = (self.g, self.xb, self.bits, self.scale, self.shift, self.coef, self.mode)
        self.g = self.xb = self.bits = self.scale = self.shift = self.coef = self.ph = self.restore = None
        self.mode = 0
        return out

    def materialize(self) -> Tensor:
        """dX through the BN's own apply kernel (the consumer could not fuse it)."""
        restore = self.restore
        g, xb, bits, scale, shift, coef, mode = self.take()
        dx = native().bn_backward_apply_coef(_to_rows(g)[0], _to_rows(xb)[0], coef, scale, shift, 1, 0.0,
                                             bits if mode == 2 else None)
        return restore(dx)


_GXF = os.environ.get("TBAMD_BN_GXF", "0") == "1"


def gxf_enabled() -> bool:
    return _GXF


class LazyAct:
    """A BatchNorm + ReLU output that is never written (csrc/xf.h): the BN forward computes its
    coefficients only and hands ``(y, scale, shift)`` to the conv that consumes it, which applies
    the transform to its activation operand (forward and weight gradient).  The BN returns a
    placeholder of the output's shape; autograd still carries the consumer's input gradient back
    to the BN backward.  ``ready`` once the BN forward has filled it."""

    __slots__ = ("y", "scale", "shift", "ph", "__weakref__")

    def __init__(self) -> None:
        self.y = self.scale = self.shift = self.ph = None

    def ready(self, a: Tensor) -> bool:
        return self.y is not None and a is self.ph


def unpack_mask(mask: Tensor, shape_like: Tensor) -> Tensor:
    """[M, C/8] mask bytes -> bool tensor shaped like ``shape_like`` (NHWC rows)."""
    bits = (mask.unsqueeze(-1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    rows, restore = _to_rows(shape_like)
    return restore(bits.reshape(rows.shape).bool())


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, training, momentum, eps, act,
                slope, stats=None, nbt=None, link=None, bn_out=None, lazy=None, gx=None):
        C = native()
        rows, restore = _to_rows(x)
        ctx.gx = gx if (gx is not None and training and x.dim() == 4) else None
        if (lazy is not None and training and stats is not None and residual is None and ACT_CODES[act] == 0
                and bn_out is None and x.dim() == 4 and rows.shape[1] % 8 == 0):
            # lazy affine output: a BN without activation whose only consumer is the residual add of
            # the BN after it (a bottleneck's downsample branch) -- coefficients only; that BN adds
            # x * scale + shift in its own apply pass, so this output is never written
            mean, invstd, scale, shift = C.bn_stats(rows, stats, weight, bias, running_mean, running_var, True,
                                                    momentum, eps, nbt)
            ctx.save_for_backward(rows, None, None, weight, mean, invstd, scale, shift, None)
            ctx.link = None
            ctx.carried = link if link is not None and link.carrier else None
            if ctx.carried is not None:
                link.ds_x, link.ds_mean = rows, mean
            ctx.bn_out = None
            ctx.cfg = (training, 0, slope, False, x.dim(), x.shape)
            ctx.restore = restore
            ctx.w_dtype = weight.dtype if weight is not None else None
            ctx.params = (weight, bias)
            ctx.orig = (x, None, eps)
            lazy.y, lazy.scale, lazy.shift = x, scale.contiguous(), shift.contiguous()
            lazy.ph = x.new_empty(1).as_strided(tuple(x.shape), (0,) * x.dim())  # shape carrier, never read
            # a WEAK back-reference: a strong one is a cycle (placeholder -> LazyAct -> placeholder) that
            # keeps this node and, through its context, the step's activations alive until a full gc
            # pass (~5 GB per ResNet-50 b256 step, tests/test_gpu_memory.py); the caller holds ``lazy``
            # until the consuming BN has run
            lazy.ph._tb_lazy_affine = weakref.ref(lazy)
            return lazy.ph
        if (lazy is not None and training and stats is not None and residual is None and ACT_CODES[act] == 1
                and bn_out is not None and x.dim() == 4 and rows.shape[1] % 8 == 0):
            # lazy output (LazyAct): coefficients only -- the consumer conv applies BN + ReLU to its
            # operand; the backward takes its ReLU mask from (x, scale, shift) and its partial sums
            # from the consumer's dgrad epilogue (bn_out, mode 1)
            mean, invstd, scale, shift = C.bn_stats(rows, stats, weight, bias, running_mean, running_var, True,
                                                    momentum, eps, nbt)
            ctx.save_for_backward(rows, None, None, weight, mean, invstd, scale, shift, None)
            ctx.link = None
            ctx.carried = None
            bn_out.mode, bn_out.xb, bn_out.mean, bn_out.scale, bn_out.shift = 1, rows, mean, scale, shift
            bn_out.bits = None
            ctx.bn_out = bn_out
            ctx.cfg = (training, 1, slope, False, x.dim(), x.shape)
            ctx.restore = restore
            ctx.w_dtype = weight.dtype if weight is not None else None
            ctx.params = (weight, bias)
            ctx.orig = (x, None, eps)
            lazy.y, lazy.scale, lazy.shift = x, scale.contiguous(), shift.contiguous()
            lazy.ph = x.new_empty(1).as_strided(tuple(x.shape), (0,) * x.dim())  # shape carrier, never read
            return lazy.ph
        code = ACT_CODES[act]
        if link is not None and link.carrier and residual is not None and link.ds_x is None:
            # carrier link whose downsample BN did not register as the mask's consumer (eval mode,
            # frozen BN, odd channel count): handing it the unmasked dy would be wrong -- the
            # residual gradient is written masked by this BN's own backward instead
            link = None
        # ReLU-after-residual keeps a 1-bit mask when its gradient goes through a link: to the
        # residual producer (ResidualGradLink) or to the consumer conv's dgrad epilogue (BnBwdLink)
        want_mask = ((link is not None or (bn_out is not None and training)) and residual is not None and code == 1
                     and rows.shape[1] % 8 == 0)
        res_rows = res_aff = None
        if residual is not None:
            lz = getattr(residual, "_tb_lazy_affine", None)
            lz = lz() if lz is not None else None
            if lz is not None and lz.ready(residual):
                # the residual is a lazy affine BN output (see above): added as y_in * scale + shift here
                # when this pass can (statistics from the conv, ReLU, mask), else materialised first
                lrows, _ = _to_rows(lz.y)
                if stats is not None and training and want_mask and lrows.dtype == x.dtype:
                    res_rows, res_aff = lrows, (lz.scale, lz.shift)
                else:
                    # (bn_apply_coeff reads rows 2 / 3 of [mean, invstd, scale, shift])
                    coeff = torch.stack([lz.scale, lz.scale, lz.scale, lz.shift]).contiguous()
                    res_rows = C.bn_apply_coeff(lrows, coeff, None, 0, 0.0, False)[0].to(x.dtype)
            else:
                res_rows, _ = _to_rows(residual.to(x.dtype))
        if stats is not None and training:
            # statistics were produced by the conv epilogue: skip the stats pass
            y, mean, invstd, scale, shift, mask = C.bn_forward_from_stats(
                rows, stats, weight, bias, running_mean, running_var, momentum, eps, res_rows, code, slope, nbt,
                want_mask, *(res_aff if res_aff is not None else (None, None)))
        else:
            y, mean, invstd, scale, shift, mask = C.bn_forward(rows, weight, bias, running_mean, running_var,
                                                               training, momentum, eps, res_rows, code, slope,
                                                               nbt if training else None, want_mask)
        keep_res = res_rows if (residual is not None and code not in (0, 1)) else None
        ctx.save_for_backward(rows, y, keep_res, weight, mean, invstd, scale, shift, mask)
        ctx.link = link if mask is not None else None
        # the downsample branch's BN (no activation, no residual): its gradient is a carrier whose
        # ReLU mask the block-output BN hands over (ResidualGradLink carrier)
        ctx.carried = (link if link is not None and link.carrier and residual is None and code == 0 and training
                       and rows.shape[1] % 8 == 0 and x.dim() == 4 else None)
        if ctx.carried is not None:
            link.ds_x, link.ds_mean = rows, mean
        ctx.bn_out = None
        if bn_out is not None and training and rows.shape[1] % 8 == 0 and x.dim() == 4:
            mode = 0
            if code == 1 and residual is None:
                mode = 1  # ReLU mask recomputed from (x, scale, shift)
            elif code == 1 and mask is not None and residual is not None:
                mode = 2  # ReLU after residual: saved bits
            elif code == 0 and residual is None:
                mode = 3
            if mode:
                bn_out.mode, bn_out.xb, bn_out.mean, bn_out.scale, bn_out.shift = mode, rows, mean, scale, shift
                bn_out.bits = mask if mode == 2 else None
                ctx.bn_out = bn_out
        ctx.cfg = (training, code, slope, residual is not None, x.dim(), x.shape)
        ctx.restore = restore
        ctx.w_dtype = weight.dtype if weight is not None else None
        ctx.params = (weight, bias)  # for the zero-copy gradient slots
        ctx.orig = (x, residual, eps)  # double-backward recompute (references, no copies)
        out = restore(y)
        if not (code == 1 and residual is not None) and out._base is not None:
            # the backward never reads y here, so the output may be modified in place
            # (stock ``nn.ReLU(inplace=True)`` after an unfused BN): hand it out as a
            # plain tensor over y's storage rather than as a view autograd would refuse
            out = out.new_empty(0).set_(y.untyped_storage(), out.storage_offset(), out.size(), out.stride())
        return out

    @staticmethod
    def backward(ctx, dy):
        if torch.is_grad_enabled():  # create_graph: differentiable ATen recompute
            return _BNActFn._backward_differentiable(ctx, dy)
        with torch.no_grad():
            return _BNActFn._backward_native(ctx, dy)

    @staticmethod
    def _backward_differentiable(ctx, dy):
        """Guarded ATen fallback for double backward (GAN gradient penalty through
        a BN discriminator): z = act(bn(x) + residual) is rebuilt with the batch
        statistics of THIS forward (saved mean / invstd in eval mode) and
        differentiated with ``create_graph``."""
        rows, y, res_rows, weight, mean, invstd, scale, shift, mask = ctx.saved_tensors
        training, code, slope, has_res, _, _ = ctx.cfg
        x, residual, eps = ctx.orig
        wp, bp = ctx.params
        if ctx.link is not None:
            ctx.link = None
        if ctx.carried is not None:  # (double backward does not use the carrier links)
            raise RuntimeError("ResidualGradLink(carrier) under create_graph: build the model without it")
        if ctx.bn_out is not None:
            ctx.bn_out.take(dy)
        shp = [1, -1] + [1] * (x.dim() - 2)
        xf = x.float()
        if training:
            dims = [0] + list(range(2, x.dim()))
            mu = xf.mean(dim=dims, keepdim=True)
            var = xf.var(dim=dims, unbiased=False, keepdim=True)
            xh = (xf - mu) * torch.rsqrt(var + eps)
        else:
            xh = (xf - mean.view(shp)) * invstd.view(shp)
        z = xh * (wp.float().view(shp) if wp is not None else 1.0) + (bp.float().view(shp) if bp is not None else 0.0)
        if residual is not None:
            z = z + residual.float()
        out = act_ref(z, {v: k for k, v in ACT_CODES.items() if isinstance(k, str)}[code], slope).to(x.dtype)
        want = [(x, ctx.needs_input_grad[0]), (wp, wp is not None and ctx.needs_input_grad[1]),
                (bp, bp is not None and ctx.needs_input_grad[2]), (residual, has_res and ctx.needs_input_grad[5])]
        ins = [t for t, need in want if need]
        grads = [None] * 17
        if ins:
            got = list(torch.autograd.grad(out, ins, dy.to(out.dtype), create_graph=True, allow_unused=True))
            for i, (t, need) in zip((0, 1, 2, 5), want):
                if need:
                    grads[i] = got.pop(0)
        return tuple(grads)

    @staticmethod
    def _backward_native(ctx, dy):
        C = native()
        rows, y, res_rows, weight, mean, invstd, scale, shift, mask = ctx.saved_tensors
        training, code, slope, has_res, _, _ = ctx.cfg
        if dy.dim() == 4:  # one layout conversion, shared by the kernel rows and the residual link
            dy = dy.contiguous(memory_format=torch.channels_last)
        dy_rows, _ = _to_rows(dy)
        wp, bp = ctx.params
        f32 = ctx.w_dtype == torch.float32
        link = ctx.link
        part = ctx.bn_out.take(dy) if ctx.bn_out is not None else None
        gs = take_slot(wp) if f32 and ctx.needs_input_grad[1] else None
        bs = take_slot(bp) if f32 and ctx.needs_input_grad[2] else None
        ev = streams.arm(dy)  # the final kernel records its completion (ops/streams.py fork)
        if part is not None and _DIAG_SKIP_BN_BWD and (not has_res or _DIAG_SKIP_BN_BWD == "all"):
            # DIAGNOSTIC ONLY (TBAMD_DIAG_SKIP_BN_BWD=inner|all, never a benchmark number): skip the
            # backward apply pass of the BNs whose partial sums came from the consumer's dgrad -- the
            # pass a consumer-side BN-backward transform ("reverse XF") would remove; dX is left
            # unwritten, so every gradient below is garbage.  Upper bound of that transform's gain.
            dx = torch.empty_like(rows)
            dg = torch.zeros_like(mean) if weight is not None else None
            db = torch.zeros_like(mean) if weight is not None else None
            dx = ctx.restore(dx)
            dres_out = None
            if link is not None:
                link.put(dy, mask)
                dres_out = dy if link.carrier else None
            elif has_res:
                dres_out = dx
            dw = dg.to(ctx.w_dtype) if weight is not None and ctx.needs_input_grad[1] else None
            dbias = db.to(ctx.w_dtype) if weight is not None and ctx.needs_input_grad[2] else None
            return dx, dw, dbias, None, None, dres_out, None, None, None, None, None, None, None, None, None, None, None
        gx, ctx.gx = ctx.gx, None
        if part is not None and gx is not None and code == 1 and rows.shape[1] % 64 == 0:
            # deferred apply (BnGradXf): the finalize only; the conv that produced x applies
            # dX = ka * mask * dy + c0 + c1 * x to its dgrad operand -- dX is never written here
            gmode = 0
            if not has_res and mask is None:
                gmode = 1  # ReLU mask recomputed from (x, scale, shift)
            elif has_res and mask is not None and link is not None and not link.carrier:
                gmode = 2  # ReLU after the residual add: saved bits; the residual gets (dy, mask)
            if gmode:
                coef, dg, db = C.bn_backward_coef(part, weight, mean, invstd, rows.shape[0], training, gs, bs)
                gx.g, gx.xb, gx.bits = dy, ctx.restore(rows), (mask if gmode == 2 else None)
                gx.scale, gx.shift, gx.coef, gx.mode, gx.restore = scale, shift, coef, gmode, ctx.restore
                gx.ph = rows.new_empty(1).view(1, 1, 1, 1).expand(ctx.cfg[5])
                streams.tag(gx.ph, ev)  # (disarm: the finalize is not the gradient's producer)
                if link is not None:
                    link.put(dy, mask)
                dw = dbias = None
                if weight is not None and ctx.needs_input_grad[1]:
                    dw = slot_alias(gs) if gs is not None else dg.to(ctx.w_dtype)
                if weight is not None and ctx.needs_input_grad[2]:
                    dbias = slot_alias(bs) if bs is not None else db.to(ctx.w_dtype)
                return (gx.ph, dw, dbias, None, None, None, None, None, None, None, None, None, None, None, None, None,
                        None)
        if part is not None:  # partial sums came from the consumer conv's dgrad epilogue
            # without a residual link the residual gradient dy * mask is written by the same pass
            own_dres = link is None and has_res
            # carrier: also the downsample BN's partial sums from this pass (its input rows / mean)
            dsx = (link.ds_x if _DS_PARTIALS and link is not None and link.carrier and link.ds_x is not None
                   and link.ds_x.shape == rows.shape and link.ds_x.dtype == rows.dtype else None)
            dx, dg, db, dres, dsp = C.bn_backward_from_partials(
                dy_rows, rows, part, weight, mean, invstd, scale, shift, training, code, slope, gs, bs,
                mask if (link is not None or own_dres) else None, own_dres,
                dsx, link.ds_mean if dsx is not None else None)
            if dsx is not None:
                link.ds_part = dsp
            if not own_dres:
                dres = None
        else:
            if y is None and code == 0:  # lazy affine output: the no-activation backward never reads y
                y = rows
            elif y is None:  # a lazy output (LazyAct) without the consumer's partials: materialise it
                y, _ = C.bn_apply_coeff(rows, torch.stack([mean, invstd, scale, shift]).contiguous(), None, code,
                                        slope, False)
            dsp = None
            if ctx.carried is not None:
                maskin, dsp = ctx.carried.take_carried(dy)
            else:
                maskin = mask if link is not None else None
            if dsp is not None:  # partial sums from the block-output BN's backward apply
                dx, dg, db, dres, _ = C.bn_backward_from_partials(dy_rows, rows, dsp, weight, mean, invstd, scale,
                                                                  shift, training, code, slope, gs, bs, maskin,
                                                                  False)
            else:
                dx, dg, db, dres = C.bn_backward(dy_rows, y, rows, res_rows, weight, mean, invstd, scale, shift,
                                                 training, code, slope, has_res, gs, bs, maskin)
        dx = ctx.restore(dx)
        streams.tag(dx, ev)
        if link is not None:  # the residual's producer applies dy * mask itself
            link.put(dy, mask)
            dres_out = dy if link.carrier else None  # carrier: the unmasked dy (see ResidualGradLink)
        else:
            dres_out = ctx.restore(dres) if has_res else None
        dw = dbias = None
        if weight is not None and ctx.needs_input_grad[1]:
            dw = slot_alias(gs) if gs is not None else dg.to(ctx.w_dtype)
        if weight is not None and ctx.needs_input_grad[2]:
            dbias = slot_alias(bs) if bs is not None else db.to(ctx.w_dtype)
        return dx, dw, dbias, None, None, dres_out, None, None, None, None, None, None, None, None, None, None, None


_DIAG_SKIP_BN_BWD = os.environ.get("TBAMD_DIAG_SKIP_BN_BWD", "")  # diagnostic (see _backward_native)

# TBAMD_DS_PARTIALS=0: the downsample BN's backward runs its own partial pass instead of taking the sums
# the block-output BN's backward apply accumulated (ResidualGradLink carrier) -- for A/B runs
_DS_PARTIALS = os.environ.get("TBAMD_DS_PARTIALS", "1") == "1"

# TBAMD_POOL_FUSED_BWD=0: the unfused backward (gather kernel writing the pool-input gradient, then
# the BN backward over it) -- for A/B runs
_POOL_FUSED_BWD = os.environ.get("TBAMD_POOL_FUSED_BWD", "1") == "1"


class _BNActPoolFn(torch.autograd.Function):
    """``maxpool(act(batch_norm(x)))`` in two kernels: statistics, then one
    fused apply + activation + max-pool pass writing the pooled tensor and a
    1-byte argmax (csrc/pool.hip); backward = argmax gather + BN backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, training, momentum, eps, act, slope, stats, nbt,
                k, s, p):
        C = native()
        rows, _ = _to_rows(x)
        code = ACT_CODES[act]
        mean, invstd, scale, shift = C.bn_stats(rows, stats if training else None, weight, bias, running_mean,
                                                running_var, training, momentum, eps, nbt if training else None)
        y, idx = C.bn_act_maxpool(x, scale, shift, code, slope, k, s, p)
        ctx.save_for_backward(rows, idx, weight, mean, invstd, scale, shift)
        ctx.cfg = (training, code, slope, k, s, p, x.shape[2], x.shape[3])
        ctx.w_dtype = weight.dtype if weight is not None else None
        ctx.params = (weight, bias)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        C = native()
        rows, idx, weight, mean, invstd, scale, shift = ctx.saved_tensors
        training, code, slope, k, s, p, H, W = ctx.cfg
        wp, bp = ctx.params
        f32 = ctx.w_dtype == torch.float32
        gs = take_slot(wp) if f32 and ctx.needs_input_grad[1] else None
        bs = take_slot(bp) if f32 and ctx.needs_input_grad[2] else None
        if _POOL_FUSED_BWD and C.bn_backward_pool_ok(H, W, rows.shape[1], k, s, p):
            # the pool-input gradient is gathered inside the BN backward passes (csrc/pool_gather.h)
            N = dy.shape[0]
            dx, dg, db = C.bn_backward_pool(dy, idx, rows, N, H, W, k, s, p, weight, mean, invstd, scale, shift,
                                            training, code, slope, gs, bs)
            Cc = rows.shape[1]

            def restore(r):
                return r.view(N, H, W, Cc).permute(0, 3, 1, 2)
        else:
            dz = C.maxpool_backward(dy, idx, H, W, k, s, p)
            dz_rows, restore = _to_rows(dz)
            # y (the BN output) is only read for a ReLU after a residual add: pass x
            dx, dg, db, _ = C.bn_backward(dz_rows, rows, rows, None, weight, mean, invstd, scale, shift, training,
                                          code, slope, False, gs, bs)
        dw = dbias = None
        if weight is not None and ctx.needs_input_grad[1]:
            dw = slot_alias(gs) if gs is not None else dg.to(ctx.w_dtype)
        if weight is not None and ctx.needs_input_grad[2]:
            dbias = slot_alias(bs) if bs is not None else db.to(ctx.w_dtype)
        return (restore(dx), dw, dbias) + (None,) * 12


def batch_norm_act(
    x: Tensor,
    weight: Optional[Tensor],
    bias: Optional[Tensor],
    running_mean: Optional[Tensor],
    running_var: Optional[Tensor],
    training: bool,
    momentum: float = 0.1,
    eps: float = 1e-5,
    residual: Optional[Tensor] = None,
    act: str = "relu",
    slope: float = 0.01,
    stats: Optional[Tensor] = None,
    num_batches_tracked: Optional[Tensor] = None,
    link: Optional[ResidualGradLink] = None,
    bn_out: Optional[BnBwdLink] = None,
    lazy: Optional[LazyAct] = None,
    gx: Optional[BnGradXf] = None,
) -> Tensor:
    """``act(batch_norm(x) + residual)`` — fused HIP path on GPU, ATen on CPU.
    ``stats``: per-tile (sum, sumsq) partials from the native conv epilogue.
    ``num_batches_tracked``: incremented by the statistics kernel (training).
    ``lazy``: return a placeholder and hand (x, scale, shift) to the consumer conv (:class:`LazyAct`)."""
    if use_native(x):
        return _BNActFn.apply(x, weight, bias, running_mean, running_var, residual, training, momentum, eps,
                              act, slope, stats, num_batches_tracked, link, bn_out, lazy, gx)
    if num_batches_tracked is not None and training:
        num_batches_tracked.add_(1)
    if running_mean is not None and running_mean.dtype != x.dtype and x.dtype != torch.float32:
        # ATen's CPU kernel wants matching dtypes: run the reference in f32
        z = F.batch_norm(x.float(), running_mean, running_var, None if weight is None else weight.float(),
                         None if bias is None else bias.float(), training, momentum, eps).to(x.dtype)
    else:
        z = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    if residual is not None:
        z = z + residual
    return act_ref(z, act, slope)


class BatchNormAct2d(nn.BatchNorm2d):
    """BatchNorm2d (+ residual add) + activation, fused into one NHWC kernel.

    ``forward(x, residual=None)``.  The affine parameters and running
    statistics stay f32 even when the module is cast to bf16/f16 (activations
    follow the input dtype; statistics are accumulated in f32/f64).
    """

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: Optional[float] = 0.1,
                 affine: bool = True, track_running_stats: bool = True, act: str = "relu",
                 slope: float = 0.01) -> None:
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        if act not in ACT_CODES:
            raise ValueError(f"unknown activation {act}")
        self.act = act
        self.slope = slope

    def _apply(self, fn, recurse=True):
        # Norm affine params and running stats stay f32 under model.to(bf16):
        # the kernel consumes f32 per-channel coefficients directly (no casts per
        # call) and the fused optimizer updates them in f32.
        super()._apply(fn, recurse)
        for name in ("weight", "bias"):
            p = getattr(self, name, None)
            if p is not None and p.is_floating_point() and p.dtype != torch.float32:
                p.data = p.data.float()
                if p.grad is not None:
                    p.grad = p.grad.float()
        for name in ("running_mean", "running_var"):
            b = getattr(self, name, None)
            if b is not None and b.dtype != torch.float32:
                setattr(self, name, b.float())
        return self

    def _check_input_dim(self, input: Tensor) -> None:
        if input.dim() < 2:
            raise ValueError(f"expected at least 2D input (got {input.dim()}D input)")

    def forward(self, x: Tensor, residual: Optional[Tensor] = None, stats: Optional[Tensor] = None,
                link: Optional[ResidualGradLink] = None, bn_out: Optional[BnBwdLink] = None,
                act: Optional[str] = None, slope: Optional[float] = None, lazy: Optional[LazyAct] = None,
                gx: Optional[BnGradXf] = None) -> Tensor:
        """``act``/``slope`` override the module's activation for this call only
        (how :func:`~torchbooster_amd.nativize` fuses a following activation
        without changing what the module computes when called on its own)."""
        self._check_input_dim(x)
        momentum = 0.0 if self.momentum is None else self.momentum
        nbt = None
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            if self.momentum is None:  # cumulative average needs the count on the host
                self.num_batches_tracked.add_(1)
                momentum = 1.0 / float(self.num_batches_tracked)
            else:  # incremented inside the statistics kernel (no extra launch)
                nbt = self.num_batches_tracked
        training = self.training or self.running_mean is None
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        return batch_norm_act(x, self.weight, self.bias, rm, rv, training, momentum, self.eps, residual,
                              self.act if act is None else act, self.slope if slope is None else slope,
                              stats if training else None, nbt, link, bn_out, lazy, gx)

    def forward_maxpool(self, x: Tensor, kernel_size: int, stride: int, padding: int,
                        stats: Optional[Tensor] = None, act: Optional[str] = None) -> Tensor:
        """``max_pool2d(act(bn(x)), kernel_size, stride, padding)`` — on GPU one
        fused apply+act+pool kernel (no full-resolution activation is written)."""
        self._check_input_dim(x)
        momentum = 0.0 if self.momentum is None else self.momentum
        nbt = None
        if self.training and self.track_running_stats and self.num_batches_tracked is not None:
            if self.momentum is None:
                self.num_batches_tracked.add_(1)
                momentum = 1.0 / float(self.num_batches_tracked)
            else:
                nbt = self.num_batches_tracked
        training = self.training or self.running_mean is None
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        act = self.act if act is None else act
        if use_native(x) and x.dim() == 4 and x.shape[1] % 8 == 0:
            return _BNActPoolFn.apply(x, self.weight, self.bias, rm, rv, training, momentum, self.eps, act,
                                      self.slope, stats, nbt, kernel_size, stride, padding)
        z = batch_norm_act(x, self.weight, self.bias, rm, rv, training, momentum, self.eps, None, act,
                           self.slope, stats if training else None, nbt)
        return F.max_pool2d(z, kernel_size, stride, padding)

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={self.act}"


class BatchNormAct1d(BatchNormAct2d):
    """Same fused kernel for (N, C) / (N, C, L) inputs."""


# --------------------------------------------------------------- GroupNorm
class _GNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, groups, eps, act, slope):
        C = native()
        N = x.shape[0]
        rows, restore = _to_rows(x)
        res_rows = _to_rows(residual.to(x.dtype))[0] if residual is not None else None
        code = ACT_CODES[act]
        y, coeff = C.gn_forward(rows, N, groups, weight, bias, eps, res_rows, code, slope)
        keep_res = res_rows if (residual is not None and code not in (0, 1)) else None
        ctx.save_for_backward(rows, y, keep_res, weight, coeff)
        ctx.cfg = (N, groups, code, slope, residual is not None)
        ctx.restore = restore
        ctx.w_dtype = weight.dtype if weight is not None else None
        ctx.params = (weight, bias)  # for the zero-copy gradient slots
        return restore(y)

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        C = native()
        rows, y, res_rows, weight, coeff = ctx.saved_tensors
        N, groups, code, slope, has_res = ctx.cfg
        dy_rows, _ = _to_rows(dy)
        gs, bs = _affine_slots(ctx, weight, 1)
        dx, dg, db, dres = C.gn_backward(dy_rows, y, rows, res_rows, weight, coeff, N, groups, code, slope, has_res,
                                         gs, bs)
        dw = _affine_grad(dg, gs, ctx.w_dtype) if weight is not None and ctx.needs_input_grad[1] else None
        dbias = _affine_grad(db, bs, ctx.w_dtype) if weight is not None and ctx.needs_input_grad[2] else None
        return ctx.restore(dx), dw, dbias, (ctx.restore(dres) if has_res else None), None, None, None, None


def group_norm_act(x: Tensor, groups: int, weight: Optional[Tensor] = None, bias: Optional[Tensor] = None,
                   eps: float = 1e-5, residual: Optional[Tensor] = None, act: str = "none",
                   slope: float = 0.01) -> Tensor:
    """``act(group_norm(x) + residual)``; InstanceNorm is ``groups == C``."""
    if use_native(x) and x.dim() >= 3:
        return _GNActFn.apply(x, weight, bias, residual, groups, eps, act, slope)
    dt = x.dtype
    z = F.group_norm(x.float(), groups, None if weight is None else weight.float(),
                     None if bias is None else bias.float(), eps).to(dt)
    if residual is not None:
        z = z + residual
    return act_ref(z, act, slope)


class GroupNormAct(nn.GroupNorm):
    """GroupNorm (+ residual) + activation in one NHWC pass; affine params stay f32."""

    def __init__(self, num_groups: int, num_channels: int, eps: float = 1e-5, affine: bool = True,
                 act: str = "none", slope: float = 0.01) -> None:
        super().__init__(num_groups, num_channels, eps, affine)
        self.act = act
        self.slope = slope

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        for name in ("weight", "bias"):
            p = getattr(self, name, None)
            if p is not None and p.is_floating_point() and p.dtype != torch.float32:
                p.data = p.data.float()
        return self

    def forward(self, x: Tensor, residual: Optional[Tensor] = None, act: Optional[str] = None,
                slope: Optional[float] = None) -> Tensor:
        return group_norm_act(x, self.num_groups, self.weight, self.bias, self.eps, residual,
                              self.act if act is None else act, self.slope if slope is None else slope)


class InstanceNormAct2d(GroupNormAct):
    """InstanceNorm2d(affine) (+ activation) == GroupNorm with one channel per group.

    Matches ``nn.InstanceNorm2d(C, affine=True)`` (no running statistics, the
    reference's setting in online.py:47 / adain.py:37)."""

    def __init__(self, num_features: int, eps: float = 1e-5, affine: bool = True, act: str = "none",
                 slope: float = 0.01) -> None:
        super().__init__(num_features, num_features, eps, affine, act, slope)


_NORM_SLOTS = os.environ.get("TBAMD_NORM_SLOTS", "1") != "0"  # 0: fresh tensors + grad-store copy (A/B)


def _affine_slots(ctx, weight: Optional[Tensor], wi: int):
    """Zero-copy gradient slots (ops/_ext.py take_slot) of an f32 affine (weight, bias) pair whose
    input indices are ``wi``, ``wi + 1``: the norm kernel's final reduction writes into them, so the
    optimizer / DDP bind step finds the gradients already in place (no per-parameter copy)."""
    if weight is None or ctx.w_dtype != torch.float32 or not _NORM_SLOTS:
        return None, None
    wp, bp = ctx.params
    gs = take_slot(wp) if ctx.needs_input_grad[wi] else None
    bs = take_slot(bp) if bp is not None and ctx.needs_input_grad[wi + 1] else None
    return (gs if gs is not None and gs.dtype == torch.float32 and gs.is_contiguous() else None,
            bs if bs is not None and bs.dtype == torch.float32 and bs.is_contiguous() else None)


def _affine_grad(g: Tensor, slot: Optional[Tensor], dt) -> Tensor:
    return slot_alias(slot) if slot is not None else g.to(dt)


# --------------------------------------------------------------- LayerNorm
class _LNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps):
        C = native()
        shape = x.shape
        rows = x.reshape(-1, shape[-1])
        res_rows = residual.reshape(-1, shape[-1]) if residual is not None else None
        y, xsum, mean, rstd = C.ln_forward(rows, res_rows, weight, bias, eps)
        xin = xsum if residual is not None else rows
        ctx.save_for_backward(xin, weight, mean, rstd)
        ctx.shape = shape
        ctx.has_res = residual is not None
        ctx.w_dtype = weight.dtype if weight is not None else None
        ctx.params = (weight, bias)  # for the zero-copy gradient slots
        ctx.set_materialize_grads(False)
        if residual is not None:
            return y.view(shape), xsum.view(shape)
        return y.view(shape), None

    @staticmethod
    @once_differentiable
    def backward(ctx, dy, dxsum):
        C = native()
        xin, weight, mean, rstd = ctx.saved_tensors
        shape = ctx.shape
        if dy is None:  # only the residual-stream output was used
            return dxsum, (dxsum if ctx.has_res else None), None, None, None
        # the residual-stream gradient is added inside the kernel (no extra pass)
        dadd = dxsum.reshape(-1, shape[-1]) if dxsum is not None else None
        gs, bs = _affine_slots(ctx, weight, 2)
        dx, dg, db = C.ln_backward(dy.reshape(-1, shape[-1]), xin, weight, mean, rstd, dadd, gs, bs)
        dx = dx.view(shape)
        dw = _affine_grad(dg, gs, ctx.w_dtype) if weight is not None and ctx.needs_input_grad[2] else None
        dbias = _affine_grad(db, bs, ctx.w_dtype) if weight is not None and ctx.needs_input_grad[3] else None
        return dx, (dx if ctx.has_res else None), dw, dbias, None


def layer_norm(x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor], eps: float = 1e-5,
               residual: Optional[Tensor] = None):
    """LayerNorm over the last dim.  With ``residual`` returns ``(ln(x + residual), x + residual)``
    (pre-norm transformer residual stream update fused into the norm)."""
    if use_native(x) and x.shape[-1] % 8 == 0 and x.shape[-1] <= 4096:
        y, xs = _LNFn.apply(x, residual, weight, bias, eps)
        return (y, xs) if residual is not None else y
    xs = x if residual is None else x + residual
    w = None if weight is None else weight.to(xs.dtype)
    b = None if bias is None else bias.to(xs.dtype)
    y = F.layer_norm(xs, (xs.shape[-1],), w, b, eps)
    return (y, xs) if residual is not None else y


class LayerNorm(nn.LayerNorm):
    """LayerNorm on the native row kernel; affine params stay f32 under dtype casts."""

    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        for name in ("weight", "bias"):
            p = getattr(self, name, None)
            if p is not None and p.is_floating_point() and p.dtype != torch.float32:
                p.data = p.data.float()
        return self

    def forward(self, x: Tensor, residual: Optional[Tensor] = None):
        return layer_norm(x, self.weight, self.bias, self.eps, residual)
