"""Put stock ``torch.nn`` models on the native MI355X kernels.

The reference builds every example model from stock modules
(/root/reference/examples/img_cls/lenet/lenet.py:29-36 ``nn.Sequential`` of
Conv2d/BatchNorm2d/GELU/MaxPool2d/Linear, the torchvision ResNet of
resnet.py:111-112, the StyleNet / AdaIN decoders of online.py:46-57 and
adain.py:36-51) and hands them to ``conf.env.make`` (config.py:174-178).
:func:`nativize` — applied by ``EnvironementConfig.make`` unless its
``native`` field is off — rewrites such a model in place so those modules run
this framework's kernels, keeping parameter objects, buffers and state-dict
keys:

1. **Leaf swaps.**  ``nn.Conv2d`` / ``nn.ConvTranspose2d`` / ``nn.Linear`` /
   ``nn.MaxPool2d`` / ``nn.ReflectionPad2d`` / nearest ``nn.Upsample`` /
   ``nn.LayerNorm`` / ``nn.BatchNorm2d`` / ``nn.GroupNorm`` become their native
   subclasses (a class swap: same object, same parameters);
   ``nn.InstanceNorm2d(affine=True)`` becomes ``InstanceNormAct2d`` sharing the
   affine parameters.  Every native module falls back to ATen on inputs its
   kernels do not take (CPU, fp32 convs, odd channel counts), so the swap never
   changes what a model computes.
2. **Fusion** (``torch.fx``): a norm whose only consumer is an activation
   (ReLU / GELU / SiLU / LeakyReLU, module or function) absorbs it; a
   BatchNorm followed by a residual add and then an activation (torchvision
   ``BasicBlock`` / ``Bottleneck`` tails) absorbs both; a Linear whose only
   consumer is an exact GELU becomes ``LinearGELU``.  The result is then an
   ``fx.GraphModule`` (same state-dict keys).  Models that do not trace keep
   the leaf swaps only.
"""
from __future__ import annotations

import logging
import operator
from typing import Dict, Optional

import torch
import torch.nn.functional as F
from torch import nn

__all__ = ["nativize", "NATIVE_TYPES"]

_LOG = logging.getLogger(__name__)


def _native_classes():
    from torchbooster_amd.ops.conv import Conv2d, ConvReLUSequential, ConvTranspose2d
    from torchbooster_amd.ops.linear import Linear, LinearGELU
    from torchbooster_amd.ops.norm import BatchNormAct2d, GroupNormAct, InstanceNormAct2d, LayerNorm
    from torchbooster_amd.ops.pool import MaxPool2d
    from torchbooster_amd.ops.resample import ReflectionPad2d, UpsampleNearest2d

    return dict(Conv2d=Conv2d, ConvTranspose2d=ConvTranspose2d, Linear=Linear, LinearGELU=LinearGELU,
                BatchNormAct2d=BatchNormAct2d, GroupNormAct=GroupNormAct, InstanceNormAct2d=InstanceNormAct2d,
                LayerNorm=LayerNorm, MaxPool2d=MaxPool2d, ReflectionPad2d=ReflectionPad2d,
                UpsampleNearest2d=UpsampleNearest2d, ConvReLUSequential=ConvReLUSequential)


def NATIVE_TYPES():
    return tuple(_native_classes().values())


def _swap_leaf(m: nn.Module, N: Dict[str, type]) -> Optional[nn.Module]:
    """Native replacement of one stock leaf module (or None to keep it)."""
    t = type(m)
    if t is nn.Conv2d:
        m.__class__ = N["Conv2d"]
        return m
    if t is nn.ConvTranspose2d:
        m.__class__ = N["ConvTranspose2d"]
        return m
    if t is nn.Linear:
        m.__class__ = N["Linear"]
        return m
    if t is nn.MaxPool2d:
        m.__class__ = N["MaxPool2d"]
        return m
    if t is nn.ReflectionPad2d:
        m.__class__ = N["ReflectionPad2d"]
        return m
    if t is nn.Upsample and m.mode == "nearest" and m.size is None:
        m.__class__ = N["UpsampleNearest2d"]
        return m
    if t is nn.LayerNorm:
        m.__class__ = N["LayerNorm"]
        m._apply(lambda x: x)  # affine params to f32 (the native kernel's coefficient dtype)
        return m
    if t is nn.BatchNorm2d:
        m.__class__ = N["BatchNormAct2d"]
        m.act, m.slope = "none", 0.01
        m._apply(lambda x: x)
        return m
    if t is nn.GroupNorm:
        m.__class__ = N["GroupNormAct"]
        m.act, m.slope = "none", 0.01
        m._apply(lambda x: x)
        return m
    if t is nn.InstanceNorm2d and m.affine and not m.track_running_stats:
        new = N["InstanceNormAct2d"](m.num_features, m.eps, True, "none")
        new.weight, new.bias = m.weight, m.bias
        new.train(m.training)
        new._apply(lambda x: x)
        return new
    return None


def _swap_all(module: nn.Module, N) -> int:
    n = 0
    for name, child in list(module.named_children()):
        new = _swap_leaf(child, N)
        if new is not None:
            if new is not child:
                setattr(module, name, new)
            n += 1
        else:
            n += _swap_all(child, N)
            n += _conv_relu_sequential(child, N)
    return n


def _conv_relu_sequential(m: nn.Module, N) -> int:
    """A plain ``nn.Sequential`` holding ``Conv2d -> ReLU`` pairs (torchvision VGG ``features``,
    the reference LeNet) becomes a :class:`~torchbooster_amd.ops.conv.ConvReLUSequential`: same
    modules, indices and state dict, the pairs run as one conv with the ReLU in its epilogue,
    decided at every forward so hooks registered later still see unfused values."""
    if type(m) is not nn.Sequential:
        return 0
    mods = list(m)
    if not any(type(a) is N["Conv2d"] and type(b) is nn.ReLU for a, b in zip(mods, mods[1:])):
        return 0
    m.__class__ = N["ConvReLUSequential"]
    return 1


_ACT_MODULES = {nn.ReLU: "relu", nn.GELU: "gelu", nn.SiLU: "silu", nn.LeakyReLU: "leaky_relu"}
_ACT_FUNCS = {F.relu: "relu", torch.relu: "relu", F.gelu: "gelu", F.silu: "silu", F.leaky_relu: "leaky_relu"}


def _act_of(node, gm) -> Optional[tuple]:
    """(act name, slope) when ``node`` is a supported elementwise activation."""
    if node.op == "call_module":
        m = gm.get_submodule(node.target)
        for cls, name in _ACT_MODULES.items():
            if type(m) is cls:
                if name == "gelu" and getattr(m, "approximate", "none") != "none":
                    return None
                return name, float(getattr(m, "negative_slope", 0.01))
        return None
    if node.op in ("call_function", "call_method"):
        if node.op == "call_method":
            tgt = {"relu": F.relu}.get(node.target)
        else:
            tgt = node.target
        if tgt in _ACT_FUNCS:
            if tgt is F.gelu and node.kwargs.get("approximate", "none") != "none":
                return None
            slope = 0.01
            if tgt is F.leaky_relu:
                slope = float(node.kwargs.get("negative_slope", node.args[1] if len(node.args) > 1 else 0.01))
            return _ACT_FUNCS[tgt], slope
    return None


def _fuse(module: nn.Module, N) -> Optional[nn.Module]:
    import torch.fx as fx

    native = NATIVE_TYPES()

    class _Tracer(fx.Tracer):
        # native modules are leaves (their forwards branch on device / dtype)
        def is_leaf_module(self, m: nn.Module, qualname: str) -> bool:
            return isinstance(m, native) or super().is_leaf_module(m, qualname)

    try:
        graph = _Tracer().trace(module)
        gm = fx.GraphModule(module, graph, type(module).__name__)
    except Exception as e:  # noqa: BLE001 - dynamic control flow etc.
        _LOG.info("nativize: %s does not trace (%s); leaf swaps only", type(module).__name__, e)
        return None
    g = gm.graph
    calls: Dict[str, int] = {}
    for n in g.nodes:
        if n.op == "call_module":
            calls[n.target] = calls.get(n.target, 0) + 1
    norm_types = (N["BatchNormAct2d"], N["GroupNormAct"])
    fused = _fold_pad_upsample(gm, calls, N)
    for n in list(g.nodes):
        if n.op != "call_module" or calls.get(n.target, 0) != 1:
            continue
        m = gm.get_submodule(n.target)
        if isinstance(m, norm_types) and getattr(m, "act", "none") in ("none", "identity", None) and len(n.users) == 1:
            u = next(iter(n.users))
            a = _act_of(u, gm)
            if a is not None and len(n.args) == 1:
                m.act, m.slope = a
                u.replace_all_uses_with(n)
                g.erase_node(u)
                fused += 1
                continue
            # bn(x) + residual -> act  ==>  bn(x, residual) with act
            if (isinstance(m, N["BatchNormAct2d"]) and u.op == "call_function"
                    and u.target in (operator.add, operator.iadd, torch.add) and len(u.users) == 1
                    and len(u.args) == 2 and not u.kwargs):
                v = next(iter(u.users))
                a = _act_of(v, gm)
                other = u.args[1] if u.args[0] is n else u.args[0]
                if a is not None and isinstance(other, fx.Node) and other is not n:
                    m.act, m.slope = a
                    with g.inserting_before(v):
                        nn_ = g.call_module(n.target, (n.args[0], other))
                    v.replace_all_uses_with(nn_)
                    g.erase_node(v)
                    g.erase_node(u)
                    g.erase_node(n)
                    fused += 1
                    continue
        if type(m) is N["Linear"] and len(n.users) == 1:
            u = next(iter(n.users))
            a = _act_of(u, gm)
            if a is not None and a[0] == "gelu":
                m.__class__ = N["LinearGELU"]
                u.replace_all_uses_with(n)
                g.erase_node(u)
                fused += 1
    if not fused:
        return None
    g.lint()
    gm.recompile()
    _LOG.info("nativize: fused %d activation / residual tails into native kernels", fused)
    return gm


def _sym_pad(m) -> Optional[int]:
    p = m.padding
    if isinstance(p, int):
        return p
    p = tuple(p)
    return p[0] if len(set(p)) == 1 else None


def _fold_pad_upsample(gm, calls: Dict[str, int], N) -> int:
    """[Upsample ->] [ReflectionPad2d ->] Conv2d  ==>  Conv2d with ``_tb_fold``."""
    g = gm.graph
    n_fold = 0
    for n in list(g.nodes):
        if n.op != "call_module" or calls.get(n.target, 0) != 1:
            continue
        conv = gm.get_submodule(n.target)
        if type(conv) is not N["Conv2d"] or getattr(conv, "_tb_fold", None) is not None or len(n.args) != 1:
            continue
        if conv.groups != 1 or tuple(conv.dilation) != (1, 1) or conv.kernel_size[0] != conv.kernel_size[1]:
            continue
        src = n.args[0]
        pad, reflect, up, drop = _sym_pad(conv) or 0, conv.padding_mode == "reflect", 1, []
        if conv.padding_mode not in ("zeros", "reflect"):
            continue

        def single(node, cls):
            if getattr(node, "op", None) != "call_module" or len(node.users) != 1 or calls.get(node.target, 0) != 1:
                return None
            m = gm.get_submodule(node.target)
            return m if isinstance(m, cls) else None

        pm = single(src, N["ReflectionPad2d"])
        if pm is not None and pad == 0 and _sym_pad(pm) is not None:
            pad, reflect = _sym_pad(pm), True
            drop.append(src)
            src = src.args[0]
        um = single(src, N["UpsampleNearest2d"])
        if um is not None and um.size is None:
            sf = um.scale_factor
            sf = sf[0] if isinstance(sf, (tuple, list)) and len(set(sf)) == 1 else sf
            if isinstance(sf, (int, float)) and float(sf).is_integer() and sf >= 1:
                up = int(sf)
                drop.append(src)
                src = src.args[0]
        if not drop:
            continue
        conv._tb_fold = (int(pad), bool(reflect), int(up))
        n.args = (src,)
        for d in drop:  # (upstream first: the pad consumed the upsample)
            if not d.users:
                g.erase_node(d)
        for d in drop[::-1]:
            if d in g.nodes and not d.users:
                g.erase_node(d)
        n_fold += 1
    return n_fold


def nativize(module: nn.Module, fuse: bool = True) -> nn.Module:
    """Rewrite ``module`` onto the native modules (see the module docstring).

    Returns the module itself (leaf swaps are in place) or, when fusions were
    applied, an ``fx.GraphModule`` over the same parameters."""
    N = _native_classes()
    new = _swap_leaf(module, N)
    if new is not None:
        return new
    _swap_all(module, N)
    if _conv_relu_sequential(module, N):
        return module  # (traced fx fusion would freeze the per-forward hook check)
    if fuse:
        gm = _fuse(module, N)
        if gm is not None:
            return gm
    return module
