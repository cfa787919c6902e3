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
2. **Fusion, per container, without changing any module's API.**  Every
   container module keeps its class, attributes and methods (``vae.decoder(z)``
   still works); what changes is the *forward of that container instance*:

   * torchvision-layout ``BasicBlock`` / ``Bottleneck`` blocks and the
     torchvision ``ResNet`` trunk get the same fused path as the in-repo
     ResNet (:mod:`torchbooster_amd.models.resnet`): conv epilogues emit the BN
     statistics, the residual add + ReLU run inside the last BN apply, the
     block input's two gradients are summed in the first conv's dgrad
     epilogue (``ResidualGradLink``), each block's output-BN backward partial
     sums come from the next block's first dgrad (``BnBwdLink``), and the stem
     BN + ReLU + max-pool is one kernel;
   * any other container whose own forward traces with ``torch.fx`` (direct
     children as leaves; no attribute stores, no ``self.training`` branch) has
     ``norm -> activation``, ``BatchNorm + residual -> activation``,
     ``Linear -> GELU`` and ``[Upsample ->] [ReflectionPad ->] Conv2d`` chains
     among its children rewritten to single native calls.

   Fused activations / pads are passed per call (``bn(x, act="relu")``,
   ``conv(x, fold=...)``), never stored on the leaf, so calling a leaf or a
   sub-container on its own computes exactly what the stock module computes.
   A fused forward falls back to the container's original forward whenever
   one of the modules it fuses has hooks (hooks registered after nativize
   still fire).
"""
from __future__ import annotations

import logging
import operator
import dis
import types
from typing import Dict, List, Optional

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
    from torchbooster_amd.ops.act import LeakyReLU

    return dict(Conv2d=Conv2d, ConvTranspose2d=ConvTranspose2d, Linear=Linear, LinearGELU=LinearGELU,
                BatchNormAct2d=BatchNormAct2d, GroupNormAct=GroupNormAct, InstanceNormAct2d=InstanceNormAct2d,
                LayerNorm=LayerNorm, MaxPool2d=MaxPool2d, ReflectionPad2d=ReflectionPad2d,
                UpsampleNearest2d=UpsampleNearest2d, ConvReLUSequential=ConvReLUSequential, LeakyReLU=LeakyReLU)


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
    if t is nn.LeakyReLU:  # (fusions into a preceding BN still see it: _act_of)
        m.__class__ = N["LeakyReLU"]
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
            if type(m) is cls or (cls is nn.LeakyReLU and type(m).__name__ == "LeakyReLU"
                                  and type(m).__module__ == "torchbooster_amd.ops.act"):
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


def _has_hooks(m: nn.Module) -> bool:
    return bool(m._forward_hooks or m._forward_pre_hooks or m._backward_hooks
                or getattr(m, "_backward_pre_hooks", None))


def forward(self, *args, **kwargs):
    """Installed as the instance forward of a nativized container: the fused
    implementation, or the class's own forward while a fused module has hooks.
    Everything is looked up through ``self`` so deep copies stay independent."""
    for name in self._tb_watch:
        if _has_hooks(self.get_submodule(name) if name else self):
            return type(self).forward(self, *args, **kwargs)
    return self._tb_impl(self, *args, **kwargs)


def _install(mod: nn.Module, impl, watched: List[str]) -> None:
    """Make ``impl(self, ...)`` this instance's forward (see :func:`forward`);
    ``watched`` are the qualified names (relative to ``mod``) of the modules
    whose hooks must still see the unfused computation."""
    object.__setattr__(mod, "_tb_impl", impl)
    object.__setattr__(mod, "_tb_watch", list(watched))
    object.__setattr__(mod, "forward", types.MethodType(forward, mod))
    object.__setattr__(mod, "_tb_nativized", True)


# ------------------------------------------------------- torchvision ResNet
def _is_conv(m, N, k: Optional[int] = None) -> bool:
    return (type(m) is N["Conv2d"] and m.bias is None and m.groups == 1 and tuple(m.dilation) == (1, 1)
            and m.padding_mode == "zeros" and not isinstance(m.padding, str)
            and (k is None or tuple(m.kernel_size) == (k, k)))


def _is_bn(m, N) -> bool:
    return type(m) is N["BatchNormAct2d"] and m.act in ("none", "identity")


def _tv_downsample(ds, N) -> bool:
    return ds is None or (type(ds) is nn.Sequential and len(ds) == 2 and _is_conv(ds[0], N, 1)
                          and _is_bn(ds[1], N))


_TV_BASIC = ("conv1", "bn1", "relu", "conv2", "bn2")
_TV_BOTTLE = ("conv1", "bn1", "conv2", "bn2", "conv3", "bn3", "relu")


def _tv_block_kind(m: nn.Module, N) -> Optional[str]:
    """"basic" / "bottleneck" for a torchvision-layout residual block."""
    kids = dict(m.named_children())
    rest = set(kids) - {"downsample"}
    if rest == set(_TV_BOTTLE):
        ok = (_is_conv(m.conv1, N, 1) and _is_conv(m.conv2, N, 3) and _is_conv(m.conv3, N, 1)
              and all(_is_bn(getattr(m, b), N) for b in ("bn1", "bn2", "bn3")))
        kind = "bottleneck"
    elif rest == set(_TV_BASIC):
        ok = _is_conv(m.conv1, N, 3) and _is_conv(m.conv2, N, 3) and _is_bn(m.bn1, N) and _is_bn(m.bn2, N)
        kind = "basic"
    else:
        return None
    if not ok or type(m.relu) is not nn.ReLU or not _tv_downsample(kids.get("downsample"), N):
        return None
    return kind


def _tv_linked(blk: nn.Module, x, bn_in=None):
    """Fused forward of a torchvision-layout block: ``(out, BnBwdLink of its output BN)``
    (the same kernel chain as :meth:`torchbooster_amd.models.resnet.Bottleneck.forward_linked`)."""
    from torchbooster_amd.models.resnet import conv_bn_act

    ds = blk.downsample
    native = x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16
    if blk._tb_kind == "basic":
        h, xp = conv_bn_act(blk.conv1, blk.bn1, x, "relu", passthrough=True)
        identity = xp if ds is None else conv_bn_act(ds[0], ds[1], xp, "none")
        return conv_bn_act(blk.conv2, blk.bn2, h, "relu", identity), None
    # bottlenecks: the in-repo model's engine itself (models/resnet.py bottleneck_linked) -- carrier,
    # lazy downsample affine, BN-in-operand and partial-sum links exactly as for models.resnet50
    from torchbooster_amd.models.resnet import bottleneck_linked

    convs = (blk.conv1, blk.conv2, blk.conv3, ds[0] if ds is not None else None)
    bns = (blk.bn1, blk.bn2, blk.bn3, ds[1] if ds is not None else None)
    acts = ("relu", "relu", "relu", "none")

    def run(i, t, residual=None, **kw):
        return conv_bn_act(convs[i], bns[i], t, acts[i], residual, **kw)

    return bottleneck_linked(x, convs, bns, run, blk.training, bn_in if native else None,
                             watch=(blk,) + ((ds,) if ds is not None else ()), acts=acts)


def _tv_block_impl(blk: nn.Module, x):
    return _tv_linked(blk, x)[0]


def _tv_trunk_impl(net: nn.Module, x):
    from torchbooster_amd.models.resnet import conv_bn_act, global_avgpool_flatten

    if net._tb_pool is not None:
        x = conv_bn_act(net.conv1, net.bn1, x, "relu", pool=net._tb_pool)
    else:
        x = net.maxpool(conv_bn_act(net.conv1, net.bn1, x, "relu"))
    link = None
    for i in range(1, 5):
        for b in getattr(net, f"layer{i}"):
            if getattr(b, "_tb_kind", None) is not None and "forward" in b.__dict__ and not any(
                    _has_hooks(b.get_submodule(n) if n else b) for n in b._tb_watch):
                x, link = _tv_linked(b, x, link)
            else:
                x, link = b(x), None
    return net.fc(global_avgpool_flatten(x, net.avgpool))


def _fuse_tv_resnet(module: nn.Module, N) -> int:
    """Fuse torchvision-layout residual blocks, and the trunk when ``module`` is a
    torchvision-layout ResNet.  Returns the number of rewritten containers."""
    n = 0
    for m in module.modules():
        if getattr(m, "_tb_nativized", False):
            continue
        kind = _tv_block_kind(m, N)
        if kind is None:
            continue
        object.__setattr__(m, "_tb_kind", kind)
        _install(m, _tv_block_impl, [""] + [k for k, _ in m.named_modules() if k])
        n += 1
    trunk = ("conv1", "bn1", "relu", "maxpool", "layer1", "layer2", "layer3", "layer4", "avgpool", "fc")
    kids = dict(module.named_children())
    if set(kids) != set(trunk) or not n:
        return n
    if not (_is_conv(module.conv1, N) and _is_bn(module.bn1, N) and type(module.relu) is nn.ReLU
            and type(module.avgpool) is nn.AdaptiveAvgPool2d and module.avgpool.output_size in (1, (1, 1))
            and type(module.fc) in (N["Linear"], nn.Linear)
            and all(type(getattr(module, f"layer{i}")) is nn.Sequential for i in range(1, 5))):
        return n
    mp = module.maxpool
    pool = None
    if type(mp) is N["MaxPool2d"] and not mp.ceil_mode and mp.dilation in (1, (1, 1)):
        k, s_, p = (v if isinstance(v, int) else v[0] for v in (mp.kernel_size, mp.stride, mp.padding))
        pool = (k, s_, p)
    object.__setattr__(module, "_tb_pool", pool)
    # the trunk's own children and layer containers; each block checks its own hooks
    _install(module, _tv_trunk_impl, ["conv1", "bn1", "relu", "maxpool", "avgpool", "fc",
                                      "layer1", "layer2", "layer3", "layer4"])
    return n + 1


# ------------------------------------------------------------ generic (fx)
_BAD_OPS = {"STORE_ATTR", "STORE_GLOBAL", "DELETE_ATTR", "DELETE_GLOBAL", "STORE_SUBSCR", "DELETE_SUBSCR"}


def _forward_is_pure(mod: nn.Module) -> bool:
    """The container's own forward stores nothing and never reads ``training``
    (a traced graph would freeze such behaviour)."""
    fwd = getattr(type(mod).forward, "__code__", None)
    if fwd is None:
        return False
    if "training" in fwd.co_names:
        return False
    return not any(ins.opname in _BAD_OPS for ins in dis.get_instructions(fwd))


def _trace(mod: nn.Module):
    import torch.fx as fx

    class _Tracer(fx.Tracer):
        def is_leaf_module(self, m: nn.Module, qualname: str) -> bool:
            return "." not in qualname  # direct children only: the container's own forward

    return fx.GraphModule(mod, _Tracer().trace(mod), type(mod).__name__)


def _fuse_container(mod: nn.Module, N) -> int:
    if getattr(mod, "_tb_nativized", False) or type(mod) is N["ConvReLUSequential"]:
        return 0
    if not list(mod.children()) or isinstance(mod, NATIVE_TYPES()):
        return 0
    if list(mod.named_parameters(recurse=False)) or list(mod.named_buffers(recurse=False)):
        return 0  # a traced copy would not follow .to() on the container's own tensors
    if type(mod).forward is nn.Module.forward or not _forward_is_pure(mod):
        return 0
    try:
        was = mod.training
        mod.training = True
        gm = _trace(mod)
        mod.training = False
        code_eval = _trace(mod).code
        mod.training = was
    except Exception as e:  # noqa: BLE001 - dynamic control flow etc.
        mod.training = was
        _LOG.debug("nativize: %s does not trace (%s)", type(mod).__name__, e)
        return 0
    if gm.code != code_eval:
        return 0
    touched: List[nn.Module] = []
    fused = _rewrite(gm, N, touched)
    if not fused:
        return 0
    gm.graph.lint()
    gm.recompile()
    names = {id(m): k for k, m in mod.named_children()}
    object.__setattr__(mod, "_tb_fused_graph", gm)
    _install(mod, _graph_impl, [names[id(m)] for m in touched if id(m) in names])
    return fused


def _graph_impl(mod: nn.Module, *args, **kwargs):
    return mod._tb_fused_graph.forward(*args, **kwargs)


def _rewrite(gm, N, touched: List[nn.Module]) -> int:
    import torch.fx as fx

    g = gm.graph
    fused = _fold_pad_upsample(gm, N, touched)
    norm_types = (N["BatchNormAct2d"], N["GroupNormAct"], N["InstanceNormAct2d"])
    for n in list(g.nodes):
        if n.op != "call_module" or n not in g.nodes:
            continue
        m = gm.get_submodule(n.target)
        if (isinstance(m, norm_types) and getattr(m, "act", "none") in ("none", "identity", None)
                and len(n.users) == 1 and len(n.args) == 1 and not n.kwargs):
            u = next(iter(n.users))
            a = _act_of(u, gm)
            if a is not None:
                n.kwargs = {"act": a[0], "slope": a[1]}
                touched += [m] + _node_modules(u, gm)
                u.replace_all_uses_with(n)
                g.erase_node(u)
                fused += 1
                continue
            # bn(x) + residual -> act  ==>  bn(x, residual, act=...)
            if (isinstance(m, N["BatchNormAct2d"]) and u.op == "call_function"
                    and u.target in (operator.add, operator.iadd, torch.add) and len(u.users) == 1
                    and len(u.args) == 2 and not u.kwargs):
                v = next(iter(u.users))
                a = _act_of(v, gm)
                other = u.args[1] if u.args[0] is n else u.args[0]
                if a is not None and isinstance(other, fx.Node) and other is not n:
                    with g.inserting_before(v):
                        nn_ = g.call_module(n.target, (n.args[0],), {"residual": other, "act": a[0],
                                                                     "slope": a[1]})
                    touched += [m] + _node_modules(v, gm)
                    v.replace_all_uses_with(nn_)
                    g.erase_node(v)
                    g.erase_node(u)
                    g.erase_node(n)
                    fused += 1
                    continue
        if type(m) is N["Linear"] and len(n.users) == 1 and len(n.args) == 1 and not n.kwargs:
            u = next(iter(n.users))
            a = _act_of(u, gm)
            if a is not None and a[0] == "gelu":
                n.kwargs = {"act": "gelu"}
                touched += [m] + _node_modules(u, gm)
                u.replace_all_uses_with(n)
                g.erase_node(u)
                fused += 1
    return fused


def _node_modules(node, gm) -> List[nn.Module]:
    return [gm.get_submodule(node.target)] if node.op == "call_module" else []


def _sym_pad(m) -> Optional[int]:
    """The padding of a conv / pad module when it is one int for every side, else None
    (``padding='same'``/``'valid'`` strings and asymmetric pads do not fold)."""
    p = m.padding
    if isinstance(p, str):
        return None
    if isinstance(p, int):
        return p
    p = tuple(p)
    return p[0] if len(p) > 0 and len(set(p)) == 1 and isinstance(p[0], int) else None


def _fold_pad_upsample(gm, N, touched: List[nn.Module]) -> int:
    """[Upsample ->] [ReflectionPad2d ->] Conv2d  ==>  conv(src, fold=(pad, reflect, up))."""
    g = gm.graph
    n_fold = 0
    for n in list(g.nodes):
        if n.op != "call_module" or n not in g.nodes:
            continue
        conv = gm.get_submodule(n.target)
        if type(conv) is not N["Conv2d"] or len(n.args) != 1 or n.kwargs:
            continue
        if conv.groups != 1 or tuple(conv.dilation) != (1, 1) or conv.kernel_size[0] != conv.kernel_size[1]:
            continue
        if conv.padding_mode not in ("zeros", "reflect"):
            continue
        own = _sym_pad(conv)
        if own is None:
            continue  # 'same' / asymmetric: the fold would drop the conv's own padding
        src = n.args[0]
        pad, reflect, up, drop = own, conv.padding_mode == "reflect", 1, []

        def single(node, cls):
            if getattr(node, "op", None) != "call_module" or len(node.users) != 1 or len(node.args) != 1:
                return None
            m = gm.get_submodule(node.target)
            return m if isinstance(m, cls) else None

        pm = single(src, N["ReflectionPad2d"])
        if pm is not None and pad == 0 and _sym_pad(pm) is not None:
            pad, reflect = _sym_pad(pm), True
            drop.append(src)
            touched.append(pm)
            src = src.args[0]
        um = single(src, N["UpsampleNearest2d"])
        if um is not None and um.size is None:
            sf = um.scale_factor
            sf = sf[0] if isinstance(sf, (tuple, list)) and len(set(sf)) == 1 else sf
            if isinstance(sf, (int, float)) and float(sf).is_integer() and sf >= 1:
                up = int(sf)
                drop.append(src)
                touched.append(um)
                src = src.args[0]
        if not drop:
            continue
        touched.append(conv)
        n.args = (src,)
        n.kwargs = {"fold": (int(pad), bool(reflect), int(up))}
        for d in drop:
            if d in g.nodes and not d.users:
                g.erase_node(d)
        for d in drop[::-1]:
            if d in g.nodes and not d.users:
                g.erase_node(d)
        n_fold += 1
    return n_fold


def nativize(module: nn.Module, fuse: bool = True) -> nn.Module:
    """Rewrite ``module`` onto the native modules (see the module docstring).

    Returns ``module`` itself (a stock leaf passed directly may come back as its
    native replacement, e.g. an ``InstanceNorm2d``): no wrapper, no GraphModule,
    same class, attributes, methods and state-dict keys."""
    N = _native_classes()
    new = _swap_leaf(module, N)
    if new is not None:
        return new
    _swap_all(module, N)
    _conv_relu_sequential(module, N)
    if fuse:
        n = _fuse_tv_resnet(module, N)
        # bottom-up: a container's fused forward treats its children as leaves
        for m in reversed(list(module.modules())):
            n += _fuse_container(m, N)
        if n:
            _LOG.info("nativize: %d container forwards rewritten onto fused native kernels", n)
    return module
