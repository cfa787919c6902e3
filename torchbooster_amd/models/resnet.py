"""ResNet family (ResNet-18/34/50/101/152), written for MI355X.

The reference pulls ``torchvision.models.resnet18`` for its img_cls example
(``/root/reference/examples/img_cls/resnet/resnet.py:111-112``); torchvision is
not part of this stack, so the architecture lives here.  The layer graph is the
standard He et al. v1.5 ResNet (stride on the 3x3 of the bottleneck) so
parameter counts match torchvision exactly (ResNet-18: 11,689,512 with a 1000
class head, ResNet-50: 25,557,032).

MI355X-specific choices:

* Every ``conv -> BN (-> ReLU)`` triple is one :class:`ConvBNAct` module, so the
  BN/activation/residual epilogue runs as ONE fused NHWC HIP kernel
  (``torchbooster_amd.ops.norm``) instead of three ATen passes over HBM.
* The residual add + final ReLU of each block is folded into the last
  ``ConvBNAct`` of the block (``residual=`` argument), which removes one more
  read+write of the activation per block.
* Models are meant to run ``channels_last`` (NHWC): the conv kernels and the
  BN kernels are all NHWC, so no layout transposes happen between them.
"""
from __future__ import annotations

import os
from typing import Tuple, Callable, List, Optional, Sequence, Type, Union

import torch
from torch import Tensor, nn

from torchbooster_amd.ops.conv import (conv2d_bn_stats, conv2d_xf_bn_stats, conv_stem, native_supported,
                                       stem_supported)
from torchbooster_amd.ops import _ext
from torchbooster_amd.ops._ext import native, use_native
from torchbooster_amd.ops.norm import BatchNormAct2d, BnBwdLink, BnGradXf, LazyAct, ResidualGradLink, gxf_enabled
from torchbooster_amd.ops.linear import Linear

__all__ = [
    "ConvBNAct",
    "conv_bn_act",
    "global_avgpool_flatten",
    "BasicBlock",
    "Bottleneck",
    "ResNet",
    "resnet18",
    "resnet34",
    "resnet50",
    "resnet101",
    "resnet152",
]


class ConvBNAct(nn.Module):
    """Conv2d (no bias) followed by a fused BatchNorm + optional residual + activation.

    ``forward(x, residual=None)`` computes ``act(bn(conv(x)) + residual)``.
    The BN/add/act part is a single fused kernel on GPU.
    """

    def __init__(
        self,
        in_ch: int,
        out_ch: int,
        kernel_size: int,
        stride: int = 1,
        padding: Optional[int] = None,
        act: str = "relu",
        groups: int = 1,
    ) -> None:
        super().__init__()
        if padding is None:
            padding = kernel_size // 2
        self.conv = nn.Conv2d(in_ch, out_ch, kernel_size, stride, padding, groups=groups, bias=False)
        self.bn = BatchNormAct2d(out_ch, act=act)

    def native_ok(self, x: Tensor) -> bool:
        """True when this conv runs through the native autograd Function."""
        c = self.conv
        return (x.is_cuda and use_native(x) and
                native_supported(x, c.weight, c.stride, c.padding, c.dilation, c.groups))

    def forward(self, x: Tensor, residual: Optional[Tensor] = None, passthrough: bool = False,
                pool: Optional[Tuple[int, int, int]] = None, link: Optional[ResidualGradLink] = None,
                bn_in: Optional[BnBwdLink] = None, bn_out: Optional[BnBwdLink] = None,
                lazy_in: Optional[LazyAct] = None, lazy_out: Optional[LazyAct] = None, gx: Optional[BnGradXf] = None):
        """``act(bn(conv(x)) + residual)``; with ``passthrough`` also returns an
        alias of ``x`` whose gradient is added by this conv's dgrad epilogue
        (hand the block input to the residual branch through it); with
        ``pool=(k, s, p)`` returns ``max_pool2d(act(bn(conv(x))), k, s, p)`` with
        the pool fused into the BN apply (the ResNet stem)."""
        return conv_bn_act(self.conv, self.bn, x, None, residual, passthrough, pool, link, bn_in, bn_out, lazy_in,
                           lazy_out, gx)


def conv_bn_act(conv: nn.Conv2d, bn: BatchNormAct2d, x: Tensor, act: Optional[str] = None,
                residual: Optional[Tensor] = None, passthrough: bool = False,
                pool: Optional[Tuple[int, int, int]] = None, link: Optional[ResidualGradLink] = None,
                bn_in: Optional[BnBwdLink] = None, bn_out: Optional[BnBwdLink] = None,
                lazy_in: Optional[LazyAct] = None, lazy_out: Optional[LazyAct] = None, gx: Optional[BnGradXf] = None):
    """The fused ``conv -> BN (+ residual) -> act`` chain on any (bias-free) conv and
    BatchNormAct2d pair: the conv epilogue emits the BN statistics, the BN apply
    takes the residual and activation, and the optional links move the residual
    gradient and the BN backward partial sums into the neighbouring dgrad
    epilogues; ``gx`` (:class:`~torchbooster_amd.ops.norm.BnGradXf`) lets the BN backward defer its
    apply into this conv's input gradient.  ``act`` overrides ``bn.act`` for this call.  Used by
    :class:`ConvBNAct` and by :func:`~torchbooster_amd.nativize` for stock
    (torchvision-layout) blocks."""
    c = conv
    if lazy_in is not None and lazy_in.ready(x):
        # x is the placeholder of a lazy BN + ReLU output: the conv applies that transform to its
        # operand (csrc/xf.h) -- the activation is never written
        assert not passthrough and pool is None
        y, stats = conv2d_xf_bn_stats(x, lazy_in.y, lazy_in.scale, lazy_in.shift, c.weight, c.stride[0],
                                      c.padding[0], bn_in, gx)
        outs = (y, stats, x)
    elif x.is_cuda and c.bias is None and native_supported(x, c.weight, c.stride, c.padding, c.dilation, c.groups):
        # native implicit-GEMM conv whose epilogue also emits the BN statistics
        # link + passthrough: this conv consumes the masked residual gradient
        outs = conv2d_bn_stats(x, c.weight, c.stride[0], c.padding[0], passthrough,
                               link if passthrough else None, bn_in, gx)
        y, stats = outs[0], outs[1]
    elif x.is_cuda and c.bias is None and stem_supported(x, c.weight, c.stride, c.padding, c.dilation, c.groups):
        # 7x7/2 stem on the native kernel (BN statistics from its epilogue)
        y, stats = conv_stem(x, c.weight)
        outs = (y, stats, x)
    else:
        y, stats = c(x), None
        outs = (y, None, x)
    if pool is not None:
        assert residual is None and not passthrough
        return bn.forward_maxpool(y, *pool, stats=stats, act=act)
    # the residual link reaches the BN that adds the residual, or (carrier) the downsample branch's BN
    bn_link = link if residual is not None or (link is not None and link.carrier and not passthrough) else None
    y = bn(y, residual, stats, bn_link, bn_out, act=act, lazy=lazy_out, gx=gx if stats is not None else None)
    return (y, outs[2]) if passthrough else y


# BN-in-operand (profiles/r04_xf/README.md): bn2 -> conv3 is never written where conv3 runs on the
# persistent 1x1 kernel (C = 64 / 128: the transform is off its critical path there) -- +0.5-0.9 %
# on the ResNet-50 step.  (Both inner BNs on every shape, the tiled-kernel variant, measured -3.4 %
# and was removed.)  TBAMD_BN_XF=0: off.
_LAZY_BN = os.environ.get("TBAMD_BN_XF", "1") != "0"
# downsample blocks: the block-output BN hands (dy, ReLU mask) to the downsample BN instead of writing
# the masked residual gradient (ops/norm.py ResidualGradLink carrier).  TBAMD_RES_CARRIER=0: off.
_RES_CARRIER = os.environ.get("TBAMD_RES_CARRIER", "1") != "0"
# downsample blocks: the downsample BN (no activation) hands its coefficients to the block-output BN,
# which adds conv_ds(x) * scale + shift itself -- the branch output is never written (ops/norm.py
# lazy affine).  TBAMD_LAZY_DS=0: off.
_LAZY_DS = os.environ.get("TBAMD_LAZY_DS", "1") != "0"


def _no_hooks(mods) -> bool:
    """No forward hook (global or on ``mods``) could see a placeholder / lazy output."""
    from torch.nn.modules import module as _mod

    if _mod._global_forward_hooks or _mod._global_forward_pre_hooks:
        return False
    return not any(m._forward_hooks or m._forward_pre_hooks for m in mods)


def _lazy_ds_ok(training: bool, down: Sequence[nn.Module], watch: Sequence[nn.Module]) -> bool:
    """The downsample branch may return a placeholder: training with autograd recording, and no
    forward hook that could see it (as _lazy_ok).  ``down`` = (conv, bn); ``watch``: wrapper modules
    whose hooks would see it too."""
    return _LAZY_DS and training and torch.is_grad_enabled() and _no_hooks(tuple(down) + tuple(watch))


def _lazy_ok(training: bool, convs: Sequence[nn.Conv2d], bns: Sequence[nn.Module],
             acts: Sequence[str], watch: Sequence[nn.Module]) -> bool:
    """The bottleneck's inner BNs can be lazy (LazyAct): training with autograd recording (the
    backward takes the mask and partial sums from the links), ReLU activations, native convs that
    the BN-in-operand kernels serve (bf16, channels % 64, at most 512 input channels), and no
    forward hook on the modules involved (it would see the placeholder).  The BN-in-operand conv is
    once-differentiable: double backward (create_graph) through such a bottleneck needs
    TBAMD_BN_XF=0."""
    if not (_LAZY_BN and training and torch.is_grad_enabled()):
        return False
    if not _no_hooks((bns[0], convs[1], bns[1], convs[2]) + tuple(watch)):
        return False
    for i in (0, 1):
        if acts[i] != "relu" or convs[i].weight.dtype != torch.bfloat16 or convs[i].out_channels % 64:
            return False
    c2, c3 = convs[1], convs[2]
    return (c2.in_channels % 64 == 0 and c2.in_channels <= 512 and c3.in_channels <= 512 and c3.out_channels % 64 == 0
            and c2.groups == 1 and c3.groups == 1)


def _gxf_ok(training: bool, convs: Sequence[Optional[nn.Conv2d]], bns: Sequence[Optional[nn.Module]],
            watch: Sequence[nn.Module]) -> bool:
    """Deferred BN backward applies (ops/norm.py BnGradXf) may run: training with autograd recording
    and no forward hook on the modules whose outputs / gradients would differ (as _lazy_ok)."""
    if not (gxf_enabled() and training and torch.is_grad_enabled()):
        return False
    return _no_hooks(tuple(m for m in tuple(convs[:3]) + tuple(bns[:3]) if m is not None) + tuple(watch))


def _gxf_pair_ok(conv: nn.Conv2d, act: str) -> bool:
    """conv -> BN + ReLU where the conv's input gradient can take the BN's apply (a bias-free 1x1
    stride-1 bf16 conv, channels on the kernel's 64-blocks)."""
    return (act == "relu" and conv.bias is None and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and conv.weight.dtype == torch.bfloat16
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def bottleneck_linked(x: Tensor, convs: Sequence[Optional[nn.Conv2d]], bns: Sequence[Optional[nn.Module]],
                      run: Callable, training: bool, bn_in: Optional[BnBwdLink] = None,
                      watch: Sequence[nn.Module] = (), acts: Sequence[str] = ("relu", "relu", "relu", "none")):
    """The fused bottleneck engine shared by the in-repo :class:`Bottleneck` and
    :func:`~torchbooster_amd.nativize`'s torchvision-layout blocks, so both get the same kernel chain.

    ``convs`` / ``bns``: conv1..conv3 and the downsample conv (None for an identity block) with their
    BatchNorms; ``run(i, x, **kw)`` runs pair ``i`` (``kw`` as :func:`conv_bn_act`: residual,
    passthrough, link, bn_in, bn_out, lazy_in, lazy_out); ``watch``: wrapper modules whose forward
    hooks must keep seeing real tensors; ``acts``: the pairs' activations (``acts[2]`` applies after
    the residual add).  Returns ``(out, BnBwdLink of the output BN)`` -- the next block's first dgrad
    computes that BN's backward partial sums (``bn_in`` is the previous block's).

    Identity blocks: the final BN keeps a 1-bit ReLU mask and hands (dy, mask) to conv1's dgrad,
    which adds dy * mask in its epilogue; downsample blocks: it hands them to the downsample BN,
    whose backward applies the mask itself (the masked residual gradient is never written)."""
    c1 = convs[0]
    has_down = convs[3] is not None
    native = (x.is_cuda and use_native(x) and c1.bias is None and
              native_supported(x, c1.weight, c1.stride, c1.padding, c1.dilation, c1.groups))
    link = None
    if (native and _RES_CARRIER and has_down and convs[2].out_channels % 8 == 0
            and torch.is_grad_enabled() and bns[2].training and bns[3].training):
        # (the block-output BN keeps its ReLU mask only for C % 8 == 0: the carrier needs it; the
        # downsample BN applies the carried mask only in training mode -- eval / frozen BNs take the
        # plain masked residual gradient)
        link = ResidualGradLink(carrier=True)
    elif native and not has_down:
        link = ResidualGradLink()
    l1, l2, l3 = (BnBwdLink(), BnBwdLink(), BnBwdLink()) if native else (None, None, None)
    # bn2 -> conv3: the BN + ReLU output is never written where conv3 runs on the persistent 1x1
    # kernel (csrc/xf.h); (bn1 -> conv2, a 3x3 on the tiled kernel, stays written: measured slower)
    z2 = None
    if native and _lazy_ok(training, convs, bns, acts, watch):
        st = convs[1].stride[0]
        npq = x.shape[0] * (-(-x.shape[2] // st)) * (-(-x.shape[3] // st))  # conv3's output pixels
        c3 = convs[2]
        if _ext.native().conv_fwd_xf_supported(npq, c3.in_channels, c3.out_channels, 1, 1, 1, 0):
            z2 = LazyAct()
    # deferred BN backward applies (BnGradXf): bn1 into conv1's input gradient, and -- in identity
    # blocks, whose output BN hands (dy, mask) to conv1 -- bn3 into conv3's
    g1 = g3 = None
    if native and _gxf_ok(training, convs, bns, watch):
        g1 = BnGradXf() if _gxf_pair_ok(convs[0], acts[0]) else None
        g3 = BnGradXf() if not has_down and link is not None and _gxf_pair_ok(convs[2], "relu") else None
    h, xp = run(0, x, passthrough=True, link=link if not has_down else None,
                bn_in=bn_in if native else None, bn_out=l1, gx=g1)
    if has_down:
        lz = LazyAct() if native and _lazy_ds_ok(training, (convs[3], bns[3]), watch) else None
        identity = run(3, xp, link=link, lazy_out=lz)
    else:
        identity = xp
    h = run(1, h, bn_in=l1, bn_out=l2, lazy_out=z2)
    return run(2, h, residual=identity, link=link, bn_in=l2, bn_out=l3, lazy_in=z2, gx=g3), l3


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_ch: int, ch: int, stride: int = 1) -> None:
        super().__init__()
        out_ch = ch * self.expansion
        self.c1 = ConvBNAct(in_ch, ch, 3, stride)
        self.c2 = ConvBNAct(ch, out_ch, 3, 1, act="relu")  # act applied after residual add
        self.down = None
        if stride != 1 or in_ch != out_ch:
            self.down = ConvBNAct(in_ch, out_ch, 1, stride, 0, act="none")

    def forward(self, x: Tensor) -> Tensor:
        h, xp = self.c1(x, passthrough=True)
        identity = xp if self.down is None else self.down(xp)
        return self.c2(h, identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_ch: int, ch: int, stride: int = 1) -> None:
        super().__init__()
        out_ch = ch * self.expansion
        self.c1 = ConvBNAct(in_ch, ch, 1, 1, 0)
        self.c2 = ConvBNAct(ch, ch, 3, stride)
        self.c3 = ConvBNAct(ch, out_ch, 1, 1, 0, act="relu")  # act after residual add
        self.down = None
        if stride != 1 or in_ch != out_ch:
            self.down = ConvBNAct(in_ch, out_ch, 1, stride, 0, act="none")

    def forward(self, x: Tensor) -> Tensor:
        # the block input reaches its second consumer through the first conv's
        # passthrough output, so its two gradients are summed inside that
        # conv's dgrad kernel instead of by a separate add
        return self.forward_linked(x)[0]

    def forward_linked(self, x: Tensor, bn_in: Optional[BnBwdLink] = None):
        """Forward that also returns the BnBwdLink of the block's output BN, so
        the next block's first conv can compute this BN's backward partial
        sums in its dgrad epilogue (``bn_in`` is the previous block's)."""
        mods = (self.c1, self.c2, self.c3, self.down)

        def run(i, t, residual=None, **kw):
            return mods[i](t, residual, **kw)

        d = self.down
        return bottleneck_linked(
            x, tuple(m.conv if m is not None else None for m in mods),
            tuple(m.bn if m is not None else None for m in mods), run, self.training, bn_in,
            watch=(self.c2, self.c3) + ((d,) if d is not None else ()),
            acts=tuple(m.bn.act if m is not None else "none" for m in mods))


Block = Union[Type[BasicBlock], Type[Bottleneck]]


class ResNet(nn.Module):
    """ResNet v1.5.

    Parameters
    ----------
    block: BasicBlock | Bottleneck
    layers: number of blocks per stage
    num_classes: classifier width
    small_input: use a 3x3/s1 stem without max-pool (CIFAR-style 32x32 input).
        The reference fine-tunes an ImageNet-stem ResNet-18 on 32x32 CIFAR
        (``resnet.py:111``), so the default is the ImageNet stem.
    zero_init_residual: zero the last BN gamma of every block (standard trick).
    """

    def __init__(
        self,
        block: Block,
        layers: Sequence[int],
        num_classes: int = 1000,
        in_ch: int = 3,
        small_input: bool = False,
        zero_init_residual: bool = False,
    ) -> None:
        super().__init__()
        self.block = block
        if small_input:
            self.stem = ConvBNAct(in_ch, 64, 3, 1, 1)
            self.pool = nn.Identity()
        else:
            self.stem = ConvBNAct(in_ch, 64, 7, 2, 3)
            self.pool = nn.MaxPool2d(3, 2, 1)
        ch = 64
        stages: List[nn.Module] = []
        for i, n in enumerate(layers):
            width = 64 * 2**i
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(block(ch, width, stride))
                ch = width * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = Linear(ch, num_classes)
        self.reset_parameters(zero_init_residual)

    def reset_parameters(self, zero_init_residual: bool = False) -> None:
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, BatchNormAct2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.c3.bn.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.c2.bn.weight)

    def features(self, x: Tensor) -> Tensor:
        if isinstance(self.pool, nn.MaxPool2d):  # BN + ReLU + max-pool fused
            p = self.pool
            x = self.stem(x, pool=(p.kernel_size, p.stride, p.padding))
        else:
            x = self.pool(self.stem(x))
        link = None
        for stage in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in stage:
                if isinstance(blk, Bottleneck):
                    # each block's output BN gets its backward partial sums from
                    # the next block's first dgrad
                    x, link = blk.forward_linked(x, link)
                else:
                    x, link = blk(x), None
        return x

    def forward(self, x: Tensor) -> Tensor:
        x = self.features(x)
        return self.fc(global_avgpool_flatten(x, self.avgpool))


def global_avgpool_flatten(x: Tensor, avgpool: nn.Module) -> Tensor:
    """``flatten(avgpool(x), 1)`` for ``AdaptiveAvgPool2d(1)``; NHWC on the native kernel."""
    if x.is_cuda and x.is_contiguous(memory_format=torch.channels_last):
        return _GlobalAvgPoolNHWC.apply(x)  # gradient born channels_last
    return torch.flatten(avgpool(x), 1)


class _GlobalAvgPoolNHWC(torch.autograd.Function):
    """``flatten(AdaptiveAvgPool2d(1)(x), 1)`` on the native NHWC pooling kernels
    (csrc/pool.hip, K7): the forward reduces HW with 16-B channel-vector loads, the
    backward writes the broadcast gradient directly in channels_last order (ATen's
    expands to NCHW and the BN backward then pays a strided layout copy of the whole
    layer4 output).  The classifier GEMM that follows runs on the native engine."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        if x.shape[1] % 8 == 0:
            return native().global_avgpool(x)
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        if C % 8 == 0:
            return native().global_avgpool_backward(dy.contiguous(), H, W)
        g = (dy * (1.0 / (H * W))).view(N, 1, 1, C).expand(N, H, W, C).contiguous()
        return g.permute(0, 3, 1, 2)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)


def resnet152(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, **kw)
