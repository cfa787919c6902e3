"""NHWC convolution: native implicit-GEMM MFMA kernels with per-shape routing.

``conv2d(x, w, bias, stride, padding)`` runs through :class:`_ConvFn` when the
shape is one the native kernels support (bf16, groups=1, dilation=1, square
kernel/stride/padding, C_in % 64 == 0, C_out % 64 == 0) and through ATen
(MIOpen) otherwise.  Inside :class:`_ConvFn` each of the three directions is
routed independently:

* forward — csrc/conv.hip (implicit GEMM, BN statistics fused in the epilogue);
* input grad — for stride 1 the same forward kernel on dY with the flipped,
  transposed weights (``conv_flip_weight``) and padding R-1-pad; strided input
  grads use MIOpen;
* weight grad — csrc/conv_wgrad.hip (split-reduction MFMA with transposing LDS
  reads and a deterministic partial-sum reduction).

Routing is autotuned per (direction, shape) the first time a shape is seen
(like ``cudnn.benchmark``: both candidates are timed with HIP events, the
faster one is cached — see :func:`autotune_table`).  ``TBAMD_CONV_AUTOTUNE=0``
always takes the native kernel; ``TBAMD_CONV_{FWD,DGRAD,WGRAD}=miopen|native``
pins one direction; ``TBAMD_NATIVE_CONV=0`` disables the native path entirely.

``passthrough=True`` additionally returns the input ``x`` as an alias whose
gradient is folded into this conv's input gradient by the dgrad epilogue
(``dx = dgrad(dY) + addend``): a ResNet block hands its input to the residual
branch through its first conv, so the residual-gradient add costs no extra
kernel (models/resnet.py).

:func:`conv2d_bn_stats` additionally returns per-tile BatchNorm partial sums
emitted by the conv epilogue (used by :class:`~torchbooster_amd.models.resnet.ConvBNAct`).
Reference: every Conv2d of the examples.
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, List, Optional, Tuple

from torchbooster_amd.ops import _agree
from torchbooster_amd.ops import convgemm as CG
from torchbooster_amd.ops import streams

import torch
from torch.autograd.function import once_differentiable
import torch.nn.functional as F
from torch import Tensor

from torchbooster_amd.ops._ext import native, slot_alias, slot_in_use, take_slot, use_native

__all__ = ["conv2d_any", "conv_any_supported", "PadConv2d", "conv2d", "conv2d_bn_stats", "conv_stem", "stem_supported", "native_supported", "conv2d_forward", "conv2d_wgrad", "autotune_table",
           "Conv2d", "ConvTranspose2d", "conv_transpose2d", "conv_transpose_supported"]

_DISABLE = os.environ.get("TBAMD_NATIVE_CONV", "1") == "0"
# DIAGNOSTIC ONLY (interference studies, never a benchmark number): skip the conv weight-gradient
# kernels of the side-stream path, leaving the gradient slots unwritten
_DIAG_SKIP_WGRAD = os.environ.get("TBAMD_DIAG_SKIP_WGRAD", "0") == "1"
# transposed convs only (A/B against MIOpen's conv_transpose2d)
_DISABLE_T = os.environ.get("TBAMD_NATIVE_CONVT", "1") == "0"
_AUTOTUNE = os.environ.get("TBAMD_CONV_AUTOTUNE", "1") != "0"
# one stderr line per autotune decision (long first steps then show progress)
_TUNE_LOG = os.environ.get("TBAMD_TUNE_LOG", "0") == "1"
_FORCE = {d: os.environ.get(f"TBAMD_CONV_{d.upper()}", "") for d in ("fwd", "dgrad", "wgrad")}
# HBM bytes/s used to price the extra BN statistics pass a MIOpen forward needs
_STATS_PASS_BW = 4.0e12

_CHOICE: Dict[tuple, str] = {}


def _tuplify(v):
    return tuple(_tuplify(x) for x in v) if isinstance(v, list) else v


# every route a table row may name (_route_choice candidates)
_ROUTE_NAMES = ("native", "miopen", "gemm", "native64", "narrow", "tinyc", "im2col", "split32", "narrow32", "tiny32",
                "tinyhalo", "splitk", "tinyin", "big256x256", "big256x128", "big128x256", "big128x128",
                "big256x256m32", "big256x128m32", "big128x256m32", "big128x128m32")

# big-tile candidates of the implicit-GEMM forward / stride-1 input gradient (csrc/conv_big.hip: 8
# waves, one workgroup per CU, (channel x pixel) tiles below, 16x16x32 MFMA, 2-4 LDS stages).  The
# per-shape A/B (profiles/r05_big) has them ahead of the 128x128 kernels by 5-19 % on the stage-3/4
# ResNet-50 shapes and behind on the early wide-pixel ones, so they are routes, not a default.
# TBAMD_CONV_BIG_ROUTES=0 drops them.
_BIG_ROUTES = os.environ.get("TBAMD_CONV_BIG_ROUTES", "1") == "1"
_BIG_CFGS = (("big256x256", (256, 256, 16, 2)), ("big256x128", (256, 128, 16, 3)),
             ("big128x256", (128, 256, 16, 2)), ("big128x128", (128, 128, 16, 4)),
             # v_mfma_f32_32x32x16_bf16 variants (round 6): same tiles, 32x32 accumulator blocks
             ("big256x256m32", (256, 256, 32, 2)), ("big256x128m32", (256, 128, 32, 3)),
             ("big128x256m32", (128, 256, 32, 3)), ("big128x128m32", (128, 128, 32, 4)))
# (the 64-channel tiles 64x256 / MF 16 and 32 lose to the shipped route on every ResNet-50 shape by
# 15-70 %, profiles/r06_m32/retime64_log.txt: not candidates)
_BIG_CODES: Dict[str, int] = {}
# tuning aid: TBAMD_CONV_RETIME=name,name,... re-times every decided route that has one of these
# candidates against them (kept only where one is faster by 3 %); with TBAMD_CONV_SAVE it writes the
# table to merge (scripts/merge_routes.py)
_RETIME = tuple(n for n in os.environ.get("TBAMD_CONV_RETIME", "").split(",") if n)
_RETIMED: set = set()


def _big_cands(K: int, C: int, make: Callable[[int], Callable[[], object]]) -> list:
    """Route candidates [(name, fn, 0.0)] for the big-tile configurations that fit K output / C
    reduction channels; ``make(code)`` returns the call with that per-call tile choice."""
    if not _BIG_ROUTES or C % 64:
        return []
    out = []
    for name, cfg in _BIG_CFGS:
        if K % cfg[0] == 0:
            code = _BIG_CODES.get(name)
            if code is None:
                code = _BIG_CODES[name] = native().conv_big_encode(*cfg)
            out.append((name, make(code), 0.0))
    return out


def load_routes(path: Optional[str] = None) -> int:
    """Seed the autotune table from a routes file (like a cuDNN/MIOpen find-db:
    decisions measured once on this GPU model, so a fresh process does not pay
    ~3 minutes of first-step timing — mostly MIOpen find of the losing
    candidates).  ``TBAMD_CONV_ROUTES`` overrides the shipped gfx950 file;
    ``TBAMD_CONV_ROUTES=none`` disables it.  Returns the number of routes."""
    import json

    path = path or os.environ.get("TBAMD_CONV_ROUTES") or os.path.join(os.path.dirname(__file__),
                                                                        "conv_routes_gfx950.json")
    if path == "none" or not os.path.exists(path):
        return 0
    with open(path) as f:
        data = json.load(f)
    n = 0
    for key, name in data.get("routes", []):
        if name in _ROUTE_NAMES:
            _CHOICE.setdefault(_tuplify(key), name)
            n += 1
    return n


def save_routes(path: str) -> None:
    """Write the current autotune table in :func:`load_routes` format."""
    import json

    rows = [json.dumps([list(_listify(k)), v]) for k, v in sorted(_CHOICE.items(), key=str)]
    with open(path, "w") as f:
        f.write('{\n"device": "gfx950",\n"routes": [\n' + ",\n".join(rows) + "\n]}\n")


def _listify(v):
    return [_listify(x) for x in v] if isinstance(v, tuple) else v


def autotune_table() -> Dict[tuple, str]:
    """(direction, shapes...) -> "native" | "miopen" decided so far."""
    return dict(_CHOICE)


if _AUTOTUNE and not _DISABLE:
    load_routes()

def _apply_occupancy_env() -> None:
    """A/B knobs: TBAMD_CONV_OCC / TBAMD_WGRAD_OCC = workgroups per CU the single-stage forward /
    weight-gradient kernels are compiled for (2, 3, 4; defaults 4 / 3)."""
    occ, wocc = os.environ.get("TBAMD_CONV_OCC"), os.environ.get("TBAMD_WGRAD_OCC")
    if not (occ or wocc) or not torch.cuda.is_available():
        return
    if occ:
        native().conv_set_occupancy(int(occ))
    if wocc:
        native().conv_wgrad_set_occupancy(int(wocc))


_apply_occupancy_env()

if os.environ.get("TBAMD_CONV_SAVE"):
    # collect this process's decisions for the shipped table (scripts/merge_routes.py)
    import atexit

    atexit.register(lambda: _CHOICE and save_routes(os.environ["TBAMD_CONV_SAVE"]))


def _pair(v) -> int:
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            return -1
        return int(v[0])
    return int(v)


def native_supported(x: Tensor, w: Tensor, stride, padding, dilation=1, groups=1) -> bool:
    if _DISABLE or not x.is_cuda or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if groups != 1 or _pair(dilation) != 1 or _pair(stride) < 1 or _pair(padding) < 0:
        return False
    if w.shape[2] != w.shape[3]:
        return False
    C, K = x.shape[1], w.shape[0]
    return C % 64 == 0 and K % 64 == 0


def _time_ms(fn: Callable[[], object], reps: int = 3) -> float:
    fn()  # warm (MIOpen runs its own find on first use)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


# TBAMD_CONV_NO_MIOPEN (default 1): never route a conv direction to MIOpen -- every shape has a
# native candidate (implicit GEMM, the phase-class strided input gradient, the generic / narrow /
# tiny-channel families, im2col + GEMM), and no first-use MIOpen find is paid.  0: MIOpen is a
# timed candidate again (taken only where it is clearly faster, _MIOPEN_MARGIN).
_NO_MIOPEN = os.environ.get("TBAMD_CONV_NO_MIOPEN", "1") == "1"

# fp32 convolutions: by default split-bf16 MFMA (three bf16 products, ~16 mantissa bits: finer than
# the TF32 PyTorch's cuDNN path may use for fp32 convs by default).  IEEE fp32 when the process asks
# for it the PyTorch way, ``torch.backends.cudnn.allow_tf32 = False`` (the switch that forbids
# reduced-precision fp32 convolutions), or with TBAMD_F32_EXACT=1: the split-bf16 candidates drop
# out and the generic kernels run the exact-f32 MFMA v_mfma_f32_16x16x4_f32 (csrc/conv_any.hip).
_F32_EXACT_ENV = os.environ.get("TBAMD_F32_EXACT", "0") == "1"
_F32_SPLIT_STATE = [None]


def f32_exact() -> bool:
    """IEEE-fp32 convolutions requested (``torch.backends.cudnn.allow_tf32 = False`` or
    TBAMD_F32_EXACT=1)."""
    return _F32_EXACT_ENV or not torch.backends.cudnn.allow_tf32


def _sync_f32_mode() -> bool:
    """Point the generic kernels' fp32 mode at :func:`f32_exact` (a host flag, set on change only);
    returns True in exact mode."""
    exact = f32_exact()
    if _F32_SPLIT_STATE[0] is not (not exact):
        native().conv_any_set_f32_split(not exact)
        _F32_SPLIT_STATE[0] = not exact
    return exact
_MIOPEN_MARGIN = float(os.environ.get("TBAMD_CONV_MIOPEN_MARGIN", "0.05"))
_MIOPEN_MARGIN_MS = float(os.environ.get("TBAMD_CONV_MIOPEN_MARGIN_MS", "0.005"))


def _route(direction: str, key: tuple, cands: List[Tuple[str, Callable[[], object], float]]):
    """Run the chosen candidate of ``cands`` [(name, fn, penalty_ms)]; the first
    candidate is the default when autotuning is off or impossible."""
    name = _route_choice(direction, key, cands)
    for n, fn, _ in cands:
        if n == name:
            return fn()
    raise RuntimeError(f"conv route {name} vanished")  # pragma: no cover


def _route_choice(direction: str, key: tuple, cands: List[Tuple[str, Callable[[], object], float]]) -> str:
    """The name of the candidate :func:`_route` runs (timing the candidates on first use)."""
    forced = _FORCE[direction]
    # deterministic mode (utils.seed / torch.use_deterministic_algorithms): MIOpen's split-K
    # solvers accumulate with float atomics (bitwise run-to-run differences on the few-pixel
    # shapes they win), every native route is fixed-order -- so native only
    if (_NO_MIOPEN or torch.are_deterministic_algorithms_enabled()) and any(c[0] != "miopen" for c in cands):
        cands = [c for c in cands if c[0] != "miopen"]
    names = [c[0] for c in cands]
    if forced in names:
        return forced
    if len(cands) == 1:
        return names[0]
    k = (direction,) + key
    name = _CHOICE.get(k)
    if name is not None and name not in names:  # a shipped / loaded route this process excludes
        name = None
    if (name is not None and _RETIME and k not in _RETIMED and not torch.cuda.is_current_stream_capturing()
            and any(n in _RETIME for n in names)):
        # tuning aid (_RETIME): the decided route against the named candidates only
        _RETIMED.add(k)
        times, cur = [], None
        best_n, best_t = None, float("inf")
        for n, fn, pen in cands:
            if n != name and n not in _RETIME:
                continue
            try:
                t = min(_time_ms(fn), _time_ms(fn)) + pen
            except RuntimeError:
                continue
            times.append(f"{n}={t:.3f}ms")
            if n == name:
                cur = t
            elif t < best_t:
                best_n, best_t = n, t
        if cur is not None and best_n is not None and best_t < cur * 0.97:
            name = best_n
            _CHOICE[k] = name
        if _TUNE_LOG:
            import sys

            print(f"[conv-retime] {k} -> {name} ({', '.join(times)})", file=sys.stderr, flush=True)
    if name is None:
        if not _AUTOTUNE or torch.cuda.is_current_stream_capturing():
            return names[0]
        times = []
        name = _agree.shared("conv", k)  # rank 0's decision (multi-rank jobs)
        if name not in names:
            best, name = float("inf"), names[0]
            mio = float("inf")
            for n, fn, pen in cands:
                try:
                    t = _time_ms(fn) + pen
                except RuntimeError as e:  # a candidate that cannot run this shape (e.g. an ATen
                    times.append(f"{n}=failed({str(e)[:60]})")  # 32-bit-index limit) drops out
                    continue
                times.append(f"{n}={t:.3f}ms")
                if n == "miopen":
                    mio = t
                elif t < best:
                    best, name = t, n
            # native first: MIOpen only where it is clearly faster (relative + absolute margin)
            if mio < best * (1.0 - _MIOPEN_MARGIN) - _MIOPEN_MARGIN_MS:
                best, name = mio, "miopen"
            _agree.publish("conv", k, name)
        else:
            times.append("rank 0's decision")
        _CHOICE[k] = name
        if _TUNE_LOG:
            import sys

            print(f"[conv-tune] {k} -> {name} ({', '.join(times)})", file=sys.stderr, flush=True)
    return name


def conv2d_forward(x: Tensor, w: Tensor, stride: int, pad: int, bias: Optional[Tensor] = None,
                   relu: bool = False) -> Tensor:
    """Raw forward on the native kernel (no autograd)."""
    return native().conv2d_fwd(x, w, bias, stride, pad, relu, False)[0]


def conv2d_wgrad(dy: Tensor, x: Tensor, kernel_size: int, stride: int, pad: int) -> Tensor:
    """Raw weight gradient on the native kernel -> [K, C, R, R] channels_last bf16."""
    return native().conv2d_wgrad(dy, x, kernel_size, kernel_size, stride, pad)


def _miopen_bwd(dy: Tensor, x: Tensor, w: Tensor, stride: int, pad: int, which: int) -> Tensor:
    mask = [which == 0, which == 1, False]
    return torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                                               mask)[which]


def _splitk_ok(x: Tensor, w: Tensor, stride: int, pad: int) -> bool:
    """bf16 conv with so few output pixels that its 128x64 tiles leave CUs idle (VGG-19 512-channel
    maps at batch 1): csrc/conv.hip conv_fwd_splitk_bf16 splits the reduction over workgroups."""
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.shape[1] % 64 or w.shape[0] % 128:
        return False
    n, _, h, wd = x.shape
    p = (h + 2 * pad - w.shape[2]) // stride + 1
    q = (wd + 2 * pad - w.shape[3]) // stride + 1
    return p > 0 and q > 0 and native().conv_fwd_splitk_ksplit(n, x.shape[1], w.shape[0], w.shape[2], w.shape[3],
                                                              p, q) > 1


def _fwd(x: Tensor, w: Tensor, bias: Optional[Tensor], stride: int, pad: int, want_stats: bool,
         relu: bool = False):
    def nat(big=-1):
        return native().conv2d_fwd(x, w, bias, stride, pad, relu, want_stats, big=big)

    def mio():
        y = F.conv2d(x, w, bias, stride, pad).contiguous(memory_format=torch.channels_last)
        return (F.relu_(y) if relu else y), None

    pen = 0.0
    if want_stats:  # a MIOpen forward leaves the BN statistics pass to the BN kernel
        n, _, h, wd = x.shape
        p = (h + 2 * pad - w.shape[2]) // stride + 1
        q = (wd + 2 * pad - w.shape[3]) // stride + 1
        pen = n * p * q * w.shape[0] * 2 / _STATS_PASS_BW * 1e3
    key = (tuple(x.shape), tuple(w.shape), stride, pad, bias is not None, want_stats) + (("relu",) if relu else ())
    cands = [("native", nat, 0.0), ("miopen", mio, pen)]
    cands += _big_cands(w.shape[0], x.shape[1], lambda code: lambda: nat(code))
    if not want_stats and CG.supported(x, w):  # explicit im2col + native GEMM (VGG-19 at batch 1)
        cands.append(("im2col", lambda: (CG.conv_fwd(x, w, bias, stride, pad, relu=relu), None), 0.0))
    if not want_stats and _splitk_ok(x, w, stride, pad):  # few output pixels: split reduction
        cands.insert(1, ("splitk", lambda: (native().conv2d_fwd_splitk(x, w, bias, stride, pad, relu), None), 0.0))
    return _route("fwd", key, cands)


class _FlipCache:
    """Flipped/transposed copies of TRAINABLE conv weights, refreshed together.

    A weight changes once per optimizer step, and every conv's dgrad of the next
    backward needs its flipped copy: instead of one small flip kernel per conv
    per backward (52 launches per ResNet-50 step), the first dgrad after a
    parameter update refreshes every registered stale copy in ONE multi-tensor
    launch (csrc/conv.hip ``flip_transpose_mt_k``).  An entry is current while
    its parameter's storage, autograd version and the fused-optimizer generation
    (ops/_ext.py ``param_generation``: native optimizer kernels write parameters
    without bumping the version counter) are unchanged."""

    def __init__(self) -> None:
        import weakref

        self._weakref = weakref.ref
        self.entries: Dict[int, list] = {}  # id(param) -> [ref, key, wt]
        self._tables: Dict[tuple, tuple] = {}  # launch tables per set of stale entries

    @staticmethod
    def _key(p: Tensor):
        from torchbooster_amd.ops._ext import param_generation

        return (p.data_ptr(), p._version, param_generation(), tuple(p.shape))

    @staticmethod
    def _shape4(p: Tensor):
        # a Linear weight [out, in] is the 1x1 conv weight [out, in, 1, 1]: its "flip" is its transpose
        return tuple(p.shape) if p.dim() == 4 else (p.shape[0], p.shape[1], 1, 1)

    def get(self, w: Tensor, owner: Tensor) -> Tensor:
        e = self.entries.get(id(owner))
        if e is not None and e[0]() is owner and e[1] == self._key(owner):
            return e[2]
        if e is None or e[0]() is not owner:
            K, C, R, S = self._shape4(owner)
            if owner.dim() == 2:
                wt = torch.empty((C, K), dtype=owner.dtype, device=owner.device)
            else:
                wt = torch.empty((C, K, R, S), dtype=owner.dtype, device=owner.device,
                                 memory_format=torch.channels_last)
            e = self.entries[id(owner)] = [self._weakref(owner), None, wt]
        self._refresh()
        return e[2]

    def _refresh(self) -> None:
        import numpy as np

        stale = []
        for pid, (ref, key, wt) in list(self.entries.items()):
            p = ref()
            if p is None:
                del self.entries[pid]
                continue
            if key != self._key(p):
                stale.append((pid, p, wt))
        if not stale:
            return
        # the shapes are part of the signature: a later parameter can reuse a dead one's id AND
        # (caching allocator) both of its addresses -- a table built for another shape would flip
        # past the end of the new copy
        sig = tuple((pid, p.data_ptr(), wt.data_ptr(), tuple(p.shape), p.dtype) for pid, p, wt in stale)
        tabs = self._tables.get(sig)
        if tabs is None:
            dev = stale[0][1].device
            rows, chunks = [], []
            for t, (_, p, wt) in enumerate(stale):
                K, C, R, S = self._shape4(p)
                rows.append([p.data_ptr(), wt.data_ptr(), K, R, S, C, 0, 0])
                for tile in range((K // 64) * (R * S * C // 64)):  # 64 x 64 tiles of [K][RSC]
                    chunks.append([t, tile, 0])
            table = torch.from_numpy(np.asarray(rows, dtype=np.int64)).to(dev)
            ck = np.asarray(chunks, dtype=np.int64)  # column 0 = (int32 tensor, int32 pad) little-endian
            tabs = (torch.from_numpy(ck).to(dev), len(chunks), table)
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[sig] = tabs
        native().conv_flip_weights_mt(*tabs)  # (entries are channels_last: [K][R][S][C] in memory)
        for pid, p, wt in stale:
            self.entries[pid][1] = self._key(p)


_FLIP_CACHE = _FlipCache()


def transposed_linear_weight(w: Tensor, owner: Tensor) -> Optional[Tensor]:
    """``owner``ᵀ ([in, out], contiguous) for a trainable bf16 Linear weight ``owner`` = ``w``'s storage,
    from the flip cache: every registered copy is refreshed in ONE launch right after each optimizer
    step (``_refresh_flipped_after_update``), so a Linear input gradient dX = dY W can run as the NT
    product dY (Wᵀ)ᵀ on the faster row-read kernel (ops/gemm.py ``mm_nn``).  None where the cache
    cannot hold it (shape not a multiple of 64, capture, frozen or non-bf16 weight)."""
    if not (owner.requires_grad and owner.dim() == 2 and owner.dtype == torch.bfloat16 and w.dtype == owner.dtype
            and owner.shape[0] % 64 == 0 and owner.shape[1] % 64 == 0 and owner.is_contiguous()
            and w.data_ptr() == owner.data_ptr() and tuple(w.shape) == tuple(owner.shape) and w.is_contiguous()
            and owner.is_cuda and not torch.cuda.is_current_stream_capturing()):
        return None
    return _FLIP_CACHE.get(w, owner)


def _refresh_flipped_after_update() -> None:
    if _FLIP_CACHE.entries:
        _FLIP_CACHE._refresh()


from torchbooster_amd.ops._ext import register_param_update_hook  # noqa: E402

register_param_update_hook(_refresh_flipped_after_update)


def _flipped(w: Tensor, owner: Optional[Tensor] = None) -> Tensor:
    """Flipped/transposed weight for the dgrad-as-forward kernel.  Frozen weights
    (a VGG feature extractor in the style-transfer examples) keep theirs cached
    on the tensor, keyed by storage and version counter, instead of re-flipping
    every backward; trainable ones go through :class:`_FlipCache` (one batched
    refresh per optimizer step).  ``owner`` is the Parameter ``w`` was taken
    from (``w`` itself may be a per-call saved-tensor object)."""
    owner = w if owner is None else owner
    if owner.requires_grad:
        if (owner.dim() == 4 and owner.shape[0] % 64 == 0 and owner.shape[1] % 64 == 0
                and w.data_ptr() == owner.data_ptr() and w.dtype == owner.dtype
                and owner.is_contiguous(memory_format=torch.channels_last)
                and not torch.cuda.is_current_stream_capturing()):
            return _FLIP_CACHE.get(w, owner)
        return native().conv_flip_weight(w)
    key = (w.data_ptr(), owner._version, tuple(w.shape))
    hit = getattr(owner, "_tb_flip", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    wt = native().conv_flip_weight(w)
    owner._tb_flip = (key, wt)
    return wt


def _dgrad(dy: Tensor, x: Tensor, w: Tensor, stride: int, pad: int, addend: Optional[Tensor],
           amask: Optional[Tensor] = None, bn_in=None, wparam: Optional[Tensor] = None) -> Tensor:
    """Input gradient (+ ``addend``, optionally masked by ``amask`` bits).

    ``bn_in`` (ops.norm.BnBwdLink): x is a BatchNorm output; the native kernel
    then also emits that BN's backward partial sums (stored on the link)."""
    R = w.shape[2]
    if addend is not None:
        addend = addend.contiguous(memory_format=torch.channels_last)
    use_bnb = bn_in is not None and bn_in.ready()

    def mio():
        dx = _miopen_bwd(dy, x, w, stride, pad, 0)
        if addend is None:
            return dx
        if amask is not None:
            from torchbooster_amd.ops.norm import unpack_mask

            return dx.add_(addend * unpack_mask(amask, addend))
        return dx.add_(addend)

    if stride in (2, 3) and amask is None and native().conv_dgrad_s2_supported(R, w.shape[3], stride):
        # stride 2 / 3: stride^2 output-phase classes of stride-1 sub-convolutions on the native
        # kernel, one launch (csrc/conv.hip conv_dgrad_s2; any padding, <= 16 taps per class)
        bnb_ok = use_bnb and addend is None  # BN partials need dX to be the BN output's whole gradient

        def nat_s2():
            wt = _flipped(w, wparam)
            if bnb_ok:
                b = bn_in
                dx, part = native().conv2d_dgrad_s2(dy, wt, R, w.shape[3], pad, x.shape[2], x.shape[3], b.mode, b.xb,
                                                    b.scale, b.shift, b.mean, b.bits, stride=stride)
                b.part, b.dx_ptr = part, dx.data_ptr()
                return dx
            dx = native().conv2d_dgrad_s2(dy, wt, R, w.shape[3], pad, x.shape[2], x.shape[3], stride=stride)[0]
            return dx if addend is None else dx.add_(addend)

        # a MIOpen dgrad leaves the BN backward its own partial pass over (dX, x)
        pen = 2 * x.numel() * x.element_size() / _STATS_PASS_BW * 1e3 if bnb_ok else 0.0
        key = (tuple(x.shape), tuple(w.shape), stride, pad, addend is not None, False, bnb_ok)
        cands = [("native", nat_s2, 0.0), ("miopen", mio, pen)]
        return _route("dgrad", key, cands)
    if not (stride == 1 and pad <= R - 1):
        # any other stride / padding: the generic native input gradient (csrc/conv_any.hip, dilated
        # dY conv + fold onto x); MIOpen is only a timed candidate (and none under the default
        # TBAMD_CONV_NO_MIOPEN=1)
        def gen():
            dx = native().conv_any_dgrad(dy, w, x.shape[2], x.shape[3], stride, pad, 1, False, _dgrad_weight(w, wparam))
            if addend is None:
                return dx
            if amask is not None:
                from torchbooster_amd.ops.norm import unpack_mask

                return dx.add_(addend * unpack_mask(amask, addend))
            return dx.add_(addend)

        key = ("generic", tuple(x.shape), tuple(w.shape), stride, pad, addend is not None, amask is not None)
        return _route("dgrad", key, [("native", gen, 0.0), ("miopen", mio, 0.0)])

    def nat(big=-1):
        wt = _flipped(w, wparam)
        if use_bnb:
            b = bn_in
            dx, part = native().conv2d_fwd(dy, wt, None, 1, R - 1 - pad, False, False, addend, amask, b.mode, b.xb,
                                           b.scale, b.shift, b.mean, b.bits, big=big)
            b.part, b.dx_ptr = part, dx.data_ptr()
            return dx
        return native().conv2d_fwd(dy, wt, None, 1, R - 1 - pad, False, False, addend, amask, big=big)[0]

    # a MIOpen dgrad leaves the BN backward its own partial pass over (dX, x)
    pen = 2 * x.numel() * x.element_size() / _STATS_PASS_BW * 1e3 if use_bnb else 0.0
    key = (tuple(x.shape), tuple(w.shape), stride, pad, addend is not None, amask is not None, use_bnb)
    cands = [("native", nat, 0.0), ("miopen", mio, pen)]
    cands += _big_cands(x.shape[1], w.shape[0], lambda code: lambda: nat(big=code))
    return _route("dgrad", key, cands)


def _wgrad(dy: Tensor, x: Tensor, w: Tensor, stride: int, pad: int, slot: Optional[Tensor] = None) -> Tensor:
    """Weight gradient; with a zero-copy ``slot`` the native kernel writes into
    it and an alias of the slot is returned (autograd adopts it as ``grad``)."""
    R = w.shape[2]

    def nat():
        if slot is not None:
            native().conv2d_wgrad(dy, x, R, R, stride, pad, slot)
            return slot_alias(slot)
        return native().conv2d_wgrad(dy, x, R, R, stride, pad)

    def mio():
        return _miopen_bwd(dy, x, w, stride, pad, 1)

    cands = [("native", nat, 0.0), ("miopen", mio, 0.0)]
    K, C = w.shape[0], w.shape[1]
    if (R == 1 and w.shape[3] == 1 and stride == 1 and pad == 0 and K % 8 == 0 and C % 8 == 0
            and dy.is_contiguous(memory_format=torch.channels_last)
            and x.is_contiguous(memory_format=torch.channels_last)):
        # a 1x1 stride-1 weight gradient IS the TN GEMM dW[K][C] = dyᵀ x over the N*H*W pixel
        # rows: the GEMM engine (csrc/gemm8.hip TN kernel among its tuned tiles) as a candidate
        def gemm():
            from torchbooster_amd.ops.gemm import mm_tn

            d2 = dy.permute(0, 2, 3, 1).reshape(-1, K)
            x2 = x.permute(0, 2, 3, 1).reshape(-1, C)
            if slot is not None:
                mm_tn(d2, x2, out=slot.permute(0, 2, 3, 1).reshape(K, C))
                return slot_alias(slot)
            return mm_tn(d2, x2).view(K, 1, 1, C).permute(0, 3, 1, 2)

        cands.insert(1, ("gemm", gemm, 0.0))
    key = (tuple(x.shape), tuple(w.shape), stride, pad)
    return _route("wgrad", key, cands)


def _gxf_conv_ok(x: Tensor, w: Tensor, stride: int, pad: int) -> bool:
    """The deferred BN apply fits this conv's input gradient: a 1x1 stride-1 unpadded bf16 conv on the
    native kernel's channel blocking (csrc/conv.hip conv_dgrad_gxf)."""
    return (w.shape[2] == 1 and w.shape[3] == 1 and stride == 1 and pad == 0 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.dim() == 4 and w.shape[0] % 64 == 0 and w.shape[1] % 64 == 0
            and not f32_exact())


def _dgrad_gxf(gx, w: Tensor, wparam: Optional[Tensor], addend: Optional[Tensor], amask: Optional[Tensor], bn_in,
               want_dz: bool):
    """(dX, dz or None): the 1x1 input gradient whose operand is the deferred BN backward apply of
    ``gx`` (ops.norm.BnGradXf); ``dz`` is that apply's result (the BN input gradient) when the
    weight gradient needs it, stored by the same kernel.  ``bn_in``: this conv's input is a BN
    output whose backward partial sums the epilogue emits (as :func:`_dgrad`)."""
    g, xb, bits, scale, shift, coef, mode = gx.take()
    wt = _flipped(w, wparam)
    if addend is not None:
        addend = addend.contiguous(memory_format=torch.channels_last)
    b = bn_in
    dx, part, dz = native().conv2d_dgrad_gxf(
        g, wt, addend, amask, b.mode if b is not None else 0, b.xb if b is not None else None,
        b.scale if b is not None else None, b.shift if b is not None else None, b.mean if b is not None else None,
        b.bits if b is not None else None, mode, xb, bits, scale, shift, coef, want_dz)
    if b is not None:
        b.part, b.dx_ptr = part, dx.data_ptr()
    return dx, (dz if want_dz else None)


def _wgrad_side(wparam: Tensor, dy: Tensor, w: Tensor, run: Callable[[Optional[Tensor]], Tensor], reads,
                fresh: bool = False) -> Tensor:
    """A weight gradient ``run(slot)`` into the parameter's zero-copy slot on the side stream (as
    :class:`_ConvFn`'s backward); ``reads``: the tensors it reads (kept alive for the side stream);
    ``fresh``: ``dy`` was produced by the kernel just issued on the compute stream."""
    slot = take_slot(wparam)
    if slot is not None and (slot.dtype != w.dtype or not slot.is_contiguous(memory_format=torch.channels_last)):
        slot = None
    if slot is not None and _DIAG_SKIP_WGRAD:
        return slot_alias(slot)  # diagnostic only: the weight gradient is NOT computed
    if slot is not None and streams.usable(dy):
        side = streams.fork(dy.device, None if fresh else dy)
        with torch.cuda.stream(side):
            dw = run(slot)
            if dw.data_ptr() != slot.data_ptr():
                slot.copy_(dw)
                dw.record_stream(side)
                dw = slot_alias(slot)
        for t in reads:
            t.record_stream(side)
        return dw
    dw = run(slot)
    if slot is None and slot_in_use(wparam) and streams.pending(dy.device):
        torch.cuda.current_stream(dy.device).wait_stream(streams.side_stream(dy.device))
    return dw


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, pad, want_stats, passthrough, link=None, bn_in=None, relu=False, gx=None):
        # relu: y = relu(conv(x) + b) from the kernel epilogue (VGG conv+ReLU pairs); the
        # backward masks dy with y > 0 before the dgrad / wgrad / bias gradient
        assert not (relu and (want_stats or passthrough)), "fused ReLU excludes stats / passthrough"
        y, stats = _fwd(x, w, bias, stride, pad, want_stats, relu)
        # no zero-filled grads for the stats / passthrough outputs (they get none)
        ctx.set_materialize_grads(False)
        ctx.relu = relu
        if relu:
            ctx.save_for_backward(x, w, y)
        else:
            ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, bias is not None)
        ctx.wparam = w  # the Parameter itself (zero-copy gradient slot lookup)
        ctx.bias_ref = bias  # (double-backward recompute only)
        ctx.link = link  # ResidualGradLink: masked residual gradient deposited by a BN backward
        ctx.bn_in = bn_in  # BnBwdLink of the BN that produced x (its partial sums come from our dgrad)
        ctx.gx = gx  # BnGradXf of the BN consuming y: its backward apply may be deferred into our dgrad
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        if passthrough:
            return y, stats, x.view_as(x)
        return y, stats

    @staticmethod
    def backward(ctx, dy, dstats, dpass=None):
        if ctx.relu and dy is not None:
            dy = dy * (ctx.saved_tensors[2] > 0).to(dy.dtype)
        if torch.is_grad_enabled():  # create_graph (e.g. a GAN gradient penalty): differentiable ATen recompute
            return _ConvFn._backward_differentiable(ctx, dy, dpass)
        with torch.no_grad():
            return _ConvFn._backward_native(ctx, dy, dpass)

    @staticmethod
    def _backward_differentiable(ctx, dy, dpass):
        """Guarded ATen fallback for double backward: rebuild y = conv(x, w) + b
        from the saved inputs and differentiate it with ``create_graph`` so the
        returned gradients carry their own graph (reference GP: gan.py:52-63)."""
        x, w = ctx.saved_tensors[:2]
        stride, pad, has_bias = ctx.cfg
        if ctx.link is not None:
            ldy, lmask = ctx.link.take()
            if ldy is not None:
                from torchbooster_amd.ops.norm import unpack_mask

                m = ldy * unpack_mask(lmask, ldy)
                dpass = m if dpass is None else dpass + m
        grads = [None] * 12
        if ctx.gx is not None:
            ctx.gx = None  # (double backward: the BN backward ran differentiably, nothing deferred)
        if dy is not None:
            b = ctx.bias_ref if has_bias else None
            ins = [t for t, need in ((x, ctx.needs_input_grad[0]), (w, ctx.needs_input_grad[1]),
                                     (b, has_bias and ctx.needs_input_grad[2])) if need]
            if ins:
                y = F.conv2d(x, w, b, stride, pad)
                got = list(torch.autograd.grad(y, ins, dy.to(y.dtype), create_graph=True, allow_unused=True))
                for i, need in enumerate((ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                                          has_bias and ctx.needs_input_grad[2])):
                    if need:
                        grads[i] = got.pop(0)
        if dpass is not None:
            grads[0] = dpass if grads[0] is None else grads[0] + dpass
        return tuple(grads)

    @staticmethod
    def _backward_native(ctx, dy, dpass):
        x, w = ctx.saved_tensors[:2]
        stride, pad, has_bias = ctx.cfg
        amask = None
        if ctx.link is not None:
            ldy, lmask = ctx.link.take()
            if ldy is not None:
                if dpass is not None:  # both forms arrived: fold the masked one in
                    from torchbooster_amd.ops.norm import unpack_mask

                    dpass = dpass + ldy * unpack_mask(lmask, ldy)
                else:
                    dpass, amask = ldy, lmask
        if dy is None:  # only the passthrough alias was used downstream
            if amask is not None:
                from torchbooster_amd.ops.norm import unpack_mask

                dpass = dpass * unpack_mask(amask, dpass)
            return dpass, None, None, None, None, None, None, None, None, None, None
        gx, ctx.gx = ctx.gx, None
        if gx is not None and gx.ready(dy):
            stride, pad, has_bias = ctx.cfg
            b = ctx.bn_in if (ctx.bn_in is not None and ctx.bn_in.ready()) else None
            add = 0 if dpass is None else (2 if amask is not None else 1)
            if (ctx.needs_input_grad[0] and not has_bias and not ctx.relu and _gxf_conv_ok(x, w, stride, pad)
                    and native().conv_dgrad_gxf_supported(gx.mode, add, b.mode if b is not None else 0)):
                dx = _dgrad_gxf(gx, w, ctx.wparam, dpass, amask, b, want_dz=ctx.needs_input_grad[1])
                dz = dx[1]
                dw = None
                if ctx.needs_input_grad[1]:
                    dw = _wgrad_side(ctx.wparam, dz, w, lambda slot: _wgrad(dz, x, w, stride, pad, slot), (dz, x),
                                     fresh=True)
                return dx[0], dw, None, None, None, None, None, None, None, None, None
            dy = gx.materialize()  # this conv cannot take the deferred apply: the BN's own kernel
        elif gx is not None and gx.mode:
            dy = gx.materialize()  # (another tensor arrived as the gradient; never expected)
        dy_in = dy
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = db = None
        if ctx.needs_input_grad[1]:
            slot = take_slot(ctx.wparam)
            if slot is not None and (slot.dtype != w.dtype or not slot.is_contiguous(memory_format=torch.channels_last)):
                slot = None
            if slot is not None and _DIAG_SKIP_WGRAD:
                dw = slot_alias(slot)  # diagnostic only: the weight gradient is NOT computed
            elif slot is not None and streams.usable(dy):
                # off the critical path: the weight gradient runs on the side stream, concurrent
                # with this dgrad and the layers below (ops/streams.py)
                main = torch.cuda.current_stream(dy.device)
                side = streams.fork(dy.device, dy if dy is dy_in else None)
                with torch.cuda.stream(side):
                    dw = _wgrad(dy, x, w, stride, pad, slot)
                    if dw.data_ptr() != slot.data_ptr():
                        # a route that returned a fresh tensor (MIOpen): land it in the slot on
                        # the side stream too -- handed out as is, the DDP reducer's bind copy or
                        # AccumulateGrad would read it on the compute stream while it is still
                        # being written here
                        slot.copy_(dw)
                        dw.record_stream(side)
                        dw = slot_alias(slot)
                dy.record_stream(side)
                x.record_stream(side)
            else:
                dw = _wgrad(dy, x, w, stride, pad, slot)
                if slot is None and slot_in_use(ctx.wparam) and streams.pending(dy.device):
                    # a second use of this weight in one backward (D(real) + D(fake), a
                    # gradient penalty, weight tying): autograd sums our fresh dw with the
                    # slot alias ON THIS STREAM, and the DDP bind copies that sum into the
                    # slot -- both must come after the side-stream kernel writing the slot
                    torch.cuda.current_stream(dy.device).wait_stream(streams.side_stream(dy.device))
        if ctx.needs_input_grad[0]:
            dx = _dgrad(dy, x, w, stride, pad, dpass, amask, ctx.bn_in, ctx.wparam)
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(dy, w.dtype)
        return dx, dw, db, None, None, None, None, None, None, None, None


class _ConvXfFn(torch.autograd.Function):
    """conv(relu(bn(y)), w) where the BN + ReLU output ``a`` is never materialised: the forward and
    the weight gradient apply ``max(y * scale + shift, 0)`` to the activation operand as it lands
    in LDS (csrc/xf.h, conv2d_fwd_xf / conv2d_wgrad_xf).  ``a_ph`` is the BN's placeholder output
    (an expanded scalar with a's shape): the input gradient w.r.t. it is the ordinary dgrad (which
    never reads the activation), so autograd still hands ``da`` to the BN backward, whose ReLU mask
    and partial sums come from ``y`` and the dgrad's BN epilogue (``bn_in``, mode 1)."""

    @staticmethod
    def forward(ctx, a_ph, y, scale, shift, w, stride, pad, bn_in=None, gx=None):
        out, stats = native().conv2d_fwd_xf(y, w, scale, shift, stride, pad, True)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(y, scale, shift, w)
        ctx.cfg = (stride, pad)
        ctx.wparam = w
        ctx.bn_in = bn_in
        ctx.gx = gx  # BnGradXf of the BN consuming out (see _ConvFn)
        ctx.mark_non_differentiable(stats)
        return out, stats

    @staticmethod
    @once_differentiable
    def backward(ctx, dy, dstats):
        if dy is None:
            return (None,) * 9
        y, scale, shift, w = ctx.saved_tensors
        stride, pad = ctx.cfg
        R = w.shape[2]
        gx, ctx.gx = ctx.gx, None
        if gx is not None and gx.ready(dy):
            b = ctx.bn_in if (ctx.bn_in is not None and ctx.bn_in.ready()) else None
            if (ctx.needs_input_grad[0] and _gxf_conv_ok(y, w, stride, pad)
                    and native().conv_dgrad_gxf_supported(gx.mode, 0, b.mode if b is not None else 0)):
                da, dz = _dgrad_gxf(gx, w, ctx.wparam, None, None, b, want_dz=ctx.needs_input_grad[4])
                dw = None
                if ctx.needs_input_grad[4]:
                    def run(slot):
                        if slot is not None:
                            native().conv2d_wgrad_xf(dz, y, scale, shift, R, R, stride, pad, slot)
                            return slot_alias(slot)
                        return native().conv2d_wgrad_xf(dz, y, scale, shift, R, R, stride, pad)

                    dw = _wgrad_side(ctx.wparam, dz, w, run, (dz, y, scale, shift), fresh=True)
                return da, None, None, None, dw, None, None, None, None
            dy = gx.materialize()
        elif gx is not None and gx.mode:
            dy = gx.materialize()
        dy_in = dy
        dy = dy.contiguous(memory_format=torch.channels_last)
        da = dw = None
        if ctx.needs_input_grad[4]:
            slot = take_slot(ctx.wparam)
            if slot is not None and (slot.dtype != w.dtype or not slot.is_contiguous(memory_format=torch.channels_last)):
                slot = None

            def wgrad():
                if slot is not None:
                    native().conv2d_wgrad_xf(dy, y, scale, shift, R, R, stride, pad, slot)
                    return slot_alias(slot)
                return native().conv2d_wgrad_xf(dy, y, scale, shift, R, R, stride, pad)

            if slot is not None and _DIAG_SKIP_WGRAD:
                dw = slot_alias(slot)  # diagnostic only: the weight gradient is NOT computed
            elif slot is not None and streams.usable(dy):
                side = streams.fork(dy.device, dy if dy is dy_in else None)
                with torch.cuda.stream(side):
                    dw = wgrad()
                for t in (dy, y, scale, shift):
                    t.record_stream(side)
            else:
                dw = wgrad()
                if slot is None and slot_in_use(ctx.wparam) and streams.pending(dy.device):
                    torch.cuda.current_stream(dy.device).wait_stream(streams.side_stream(dy.device))
        if ctx.needs_input_grad[0]:
            # the dgrad needs only a's shape (and the BN link for its epilogue partials)
            da = _dgrad(dy, y, w, stride, pad, None, None, ctx.bn_in, ctx.wparam)
        return da, None, None, None, dw, None, None, None, None


def xf_supported(y: Tensor, w: Tensor, stride, padding) -> bool:
    """The BN-in-operand conv path (csrc/xf.h): bf16 NHWC, C % 64 == K % 64 == 0, C <= 512, square taps,
    groups 1, the single-stage forward addressing (any stride / zero padding)."""
    return (y.is_cuda and y.dim() == 4 and y.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and y.shape[1] % 64 == 0 and y.shape[1] <= 512 and w.shape[0] % 64 == 0 and w.shape[1] == y.shape[1]
            and w.shape[2] == w.shape[3] and _pair(stride) >= 1 and _pair(padding) >= 0 and not _DISABLE
            and use_native(y))


def conv2d_xf_bn_stats(a_ph: Tensor, y: Tensor, scale: Tensor, shift: Tensor, w: Tensor, stride: int, padding: int,
                       bn_in=None, gx=None):
    """``(conv(relu(y * scale + shift), w), bn_partials)`` without materialising the activation
    (see :class:`_ConvXfFn`); ``a_ph`` is the placeholder the producing BN returned."""
    w = w.contiguous(memory_format=torch.channels_last)
    return _ConvXfFn.apply(a_ph, y.contiguous(memory_format=torch.channels_last), scale, shift, w, _pair(stride),
                           _pair(padding), bn_in, gx)


def conv2d(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, stride=1, padding=0, dilation=1,
           groups=1, relu: bool = False) -> Tensor:
    """``conv2d`` (``relu``: followed by ReLU, fused into the native kernel's epilogue)."""
    if use_native(x) and native_supported(x, w, stride, padding, dilation, groups):
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
        return _ConvFn.apply(x, w, bias, _pair(stride), _pair(padding), False, False, None, None, relu)[0]
    y = F.conv2d(x, w, bias, stride, padding, dilation, groups)
    return F.relu(y) if relu else y


def stem_supported(x: Tensor, w: Tensor, stride, padding, dilation=1, groups=1) -> bool:
    """The ResNet 7x7/2 stem on 3-channel bf16 images (csrc/conv.hip ``conv_stem_fwd``)."""
    return (x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and tuple(w.shape[1:]) == (3, 7, 7) and w.shape[0] % 64 == 0
            and _pair(stride) == 2 and _pair(padding) == 3 and _pair(dilation) == 1 and groups == 1
            and not _DISABLE and use_native(x))


def _pack_stem_w(w: Tensor) -> Tensor:
    """[K, 3, 7, 7] -> [K, 256]: window row r holds (tap s, channel c) at r*32 + s*4 + c, zero padded."""
    K = w.shape[0]
    wp = w.new_zeros(K, 8, 8, 4)
    wp[:, :7, :7, :3] = w.permute(0, 2, 3, 1)
    return wp.reshape(K, 256)


class _StemConvFn(torch.autograd.Function):
    """ResNet stem on the native kernels — forward (BN statistics from its
    epilogue) and weight gradient both read the pre-padded 4-channel image
    (csrc/conv.hip ``conv_stem_*``); each direction is autotuned against MIOpen."""

    @staticmethod
    def forward(ctx, x, w, want_stats):
        H, W = x.shape[2], x.shape[3]
        keep = {}

        def nat():
            xp = native().conv2d_stem_pad(x)
            keep["xp"] = xp
            y, st = native().conv2d_stem_fwd(xp, _pack_stem_w(w), H, W, want_stats)
            return y, (st if want_stats else None)

        def mio():
            return F.conv2d(x, w, None, 2, 3).contiguous(memory_format=torch.channels_last), None

        pen = 0.0
        if want_stats:
            n = x.shape[0]
            pen = n * ((H - 1) // 2 + 1) * ((W - 1) // 2 + 1) * w.shape[0] * 2 / _STATS_PASS_BW * 1e3
        y, stats = _route("fwd", ("stem", tuple(x.shape), tuple(w.shape), want_stats),
                          [("native", nat, 0.0), ("miopen", mio, pen)])
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x, w)
        ctx.xp = keep.get("xp")  # the padded image, reused by the native weight gradient
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    @once_differentiable
    def backward(ctx, dy, dstats):
        x, w = ctx.saved_tensors
        dx = dw = None
        if dy is None:
            return None, None, None
        if ctx.needs_input_grad[0]:
            dx = _miopen_bwd(dy, x, w, 2, 3, 0)
        if ctx.needs_input_grad[1]:
            K, H, W = w.shape[0], x.shape[2], x.shape[3]
            cl = w.is_contiguous(memory_format=torch.channels_last)

            def nat():
                xp = ctx.xp if ctx.xp is not None else native().conv2d_stem_pad(x)
                g = native().conv2d_stem_wgrad(dy, xp, H, W).view(K, 8, 8, 4)[:, :7, :7, :3].permute(0, 3, 1, 2)
                return g.contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format)

            def mio():
                return _miopen_bwd(dy, x, w, 2, 3, 1)

            dw = _route("wgrad", ("stem", tuple(x.shape), tuple(w.shape)), [("native", nat, 0.0), ("miopen", mio, 0.0)])
        ctx.xp = None
        return dx, dw, None


def conv_stem(x: Tensor, w: Tensor, want_stats: bool = True):
    """ResNet stem conv ``(y, bn_partials_or_None)`` (see :class:`_StemConvFn`)."""
    x = x.contiguous(memory_format=torch.channels_last)
    return _StemConvFn.apply(x, w, want_stats)


def conv2d_bn_stats(x: Tensor, w: Tensor, stride: int, padding: int, passthrough: bool = False, link=None,
                    bn_in=None, gx=None):
    """Conv returning ``(y, bn_partials_or_None[, x_alias])``.

    ``bn_partials`` are the epilogue's per-tile channel sums (None when the conv
    ran on MIOpen); with ``passthrough`` the third output is an alias of ``x``
    whose gradient is fused into this conv's dgrad."""
    if use_native(x) and native_supported(x, w, stride, padding):
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
        return _ConvFn.apply(x, w, None, _pair(stride), _pair(padding), True, passthrough, link, bn_in, False, gx)
    y = F.conv2d(x, w, None, stride, padding)
    return (y, None, x) if passthrough else (y, None)


# ------------------------------------------------------------ generic convolution
def conv_any_supported(x: Tensor, w: Tensor, stride, padding, dilation=1, groups=1) -> bool:
    """csrc/conv_any.hip: any channel counts, square taps / stride / padding, bf16 or
    fp32 (reference precision), groups 1, no dilation."""
    if _DISABLE or not x.is_cuda or x.dim() != 4 or x.dtype not in (torch.bfloat16, torch.float32):
        return False
    if w.dtype != x.dtype or groups != 1 or _pair(dilation) != 1 or w.shape[2] != w.shape[3]:
        return False
    return _pair(stride) >= 1 and _pair(padding) >= 0 and use_native(x)


def _virtual(x: Tensor, pad: int, up: int, reflect: bool) -> Tensor:
    """pad(upsample(x)) materialised (the MIOpen candidate and the double-backward path)."""
    if up > 1:
        x = F.interpolate(x, scale_factor=up, mode="nearest")
    if pad:
        x = F.pad(x, (pad,) * 4, mode="reflect" if reflect else "constant")
    return x


def _bias_grad(dy: Tensor, dtype: torch.dtype) -> Tensor:
    """sum over (N, H, W) of a channels_last dy on the native column-sum kernel
    (csrc/colsum.hip); C % 8 != 0 sums G rows at once as one row of G*C columns."""
    C = dy.shape[1]
    rows = dy.permute(0, 2, 3, 1)
    if dy.is_cuda and rows.is_contiguous() and dy.dtype in (torch.bfloat16, torch.float32) and not _DISABLE:
        G = 8 // math.gcd(C, 8)
        M = rows.numel() // C
        if M % G == 0 and M > 0:
            s = native().colsum(rows.reshape(M // G, G * C), None)
            return (s.view(G, C).float().sum(0) if G > 1 else s).to(dtype)
    return dy.float().sum(dim=(0, 2, 3)).to(dtype)


def _dgrad_weight(w: Tensor, owner: Optional[Tensor]) -> Optional[Tensor]:
    """Cached flipped transpose for the generic dgrad (bf16; fp32 flips inside the op)."""
    if w.dtype != torch.bfloat16 or not w.is_contiguous(memory_format=torch.channels_last):
        return None
    return _flipped(w, owner)


def _virt64_ok(x: Tensor, w: Tensor, stride: int, up: int) -> bool:
    """csrc/conv.hip VIRT kernels: bf16, C % 64 == K % 64 == 0, upsample 1/2/4, square taps,
    stride 1 or 2 (the dgrad kernels' strides)."""
    return (x.dtype == torch.bfloat16 and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0 and up in (1, 2, 4)
            and stride in (1, 2) and w.shape[2] == w.shape[3] and w.is_contiguous(memory_format=torch.channels_last))


def _virt_wgrad_ok(x: Tensor, w: Tensor, stride: int, up: int) -> bool:
    """csrc/conv_wgrad.hip conv_wgrad_virtual: as _virt64_ok, and K % 32 == 0 outputs (32-row dY
    tiles: the StyleNet 64 -> 32 upsampling conv, ref examples/img_stt/online/online.py:48 DeconvIN)."""
    return (x.dtype == torch.bfloat16 and x.shape[1] % 64 == 0 and w.shape[0] % 32 == 0 and up in (1, 2, 4)
            and stride in (1, 2) and w.shape[2] == w.shape[3])


def _narrow_ok(x: Tensor, w: Tensor, stride: int, pad: int, up: int, reflect: bool) -> bool:
    """csrc/conv_narrow.hip: bf16, C in {32, 64}, K <= 16 output channels, taps <= 9x9, stride 1
    (the RGB heads of the style-transfer decoders, reference adain.py:51 / online.py:57)."""
    C, K, R, S = x.shape[1], w.shape[0], w.shape[2], w.shape[3]
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and C in (32, 64) and 1 <= K <= 16
            and R <= 9 and S <= 9 and stride == 1 and up in (1, 2, 4)
            and (not reflect or (pad < x.shape[2] * up and pad < x.shape[3] * up)))


def _tinyc_ok(x: Tensor, w: Tensor, stride: int, pad: int, up: int, reflect: bool) -> bool:
    """csrc/conv_narrow.hip conv_tinyc_fwd: bf16, C*R*S <= 256 reduction taps (RGB / grey input
    convs: VGG 3->64, DCGAN discriminator input, StyleNet 3->32 9x9, LeNet), K % 16 == 0."""
    C, K, R, S = x.shape[1], w.shape[0], w.shape[2], w.shape[3]
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and C * R * S <= 256 and K % 16 == 0
            and up == 1 and stride >= 1 and (not reflect or (pad < x.shape[2] and pad < x.shape[3])))


def _narrow32_ok(x: Tensor, w: Tensor, stride: int, pad: int, up: int, reflect: bool) -> bool:
    """csrc/conv_narrow.hip conv_narrow_fwd32: the halo-tile kernel at fp32 (three split-bf16 runs)."""
    C, K, R, S = x.shape[1], w.shape[0], w.shape[2], w.shape[3]
    return (not f32_exact() and x.dtype == torch.float32 and w.dtype == torch.float32 and C in (32, 64) and 1 <= K <= 16
            and R <= 9 and S <= 9 and stride == 1 and up in (1, 2, 4) and x.numel() % 4 == 0
            and (not reflect or (pad < x.shape[2] * up and pad < x.shape[3] * up)))


def _tiny32_ok(x: Tensor, w: Tensor, stride: int, pad: int, up: int, reflect: bool) -> bool:
    """csrc/conv_narrow.hip conv_tiny32_fwd: the tiny-channel gather kernel at fp32 (split-bf16),
    e.g. StyleNet's 9x9 3->32 input conv at the reference precision."""
    C, K, R, S = x.shape[1], w.shape[0], w.shape[2], w.shape[3]
    return (not f32_exact() and x.dtype == torch.float32 and w.dtype == torch.float32 and C * R * S <= 256
            and K % 16 == 0
            and up == 1 and stride >= 1 and (not reflect or (pad < x.shape[2] and pad < x.shape[3])))


def _tinyhalo_ok(x: Tensor, w: Tensor, stride: int, pad: int, up: int, reflect: bool) -> bool:
    """csrc/conv_narrow.hip conv_tinyhalo_fwd: stride-1 conv with C <= 4 input channels from an LDS
    halo tile (bf16, or fp32 as split-bf16), taps <= 9x9, K % 16 == 0."""
    C, K, R, S = x.shape[1], w.shape[0], w.shape[2], w.shape[3]
    return ((x.dtype == torch.bfloat16 or (x.dtype == torch.float32 and not f32_exact())) and w.dtype == x.dtype
            and 1 <= C <= 4 and K % 16 == 0
            and R <= 9 and S <= 9 and stride == 1 and up == 1
            and (not reflect or (pad < x.shape[2] and pad < x.shape[3])))


def _window_gemm(x: Tensor, w: Tensor, b: Optional[Tensor]) -> Tensor:
    """A conv whose window covers the whole (unpadded) input — 1x1 output, e.g. a DCGAN
    discriminator head 1024x4x4 -> 1 — is one GEMM over the flattened NHWC rows."""
    N, K = x.shape[0], w.shape[0]
    a = x.permute(0, 2, 3, 1).reshape(N, -1)
    wf = w.permute(0, 2, 3, 1).reshape(K, -1)
    from torchbooster_amd.ops import gemm as G

    if G.supported_nt(a, wf) and (b is None or b.is_cuda):
        # the native GEMM (bias in its epilogue; the 1-column head is padded to 8 columns)
        y = G.mm_nt(a, wf, bias=None if b is None else b.to(x.dtype), blas=False)
    else:
        y = torch.addmm(b.to(x.dtype), a, wf.t()) if b is not None else a @ wf.t()
    return y.view(N, K, 1, 1)


def _relu(y: Tensor) -> Tensor:
    """ReLU after a conv that could not take it in its epilogue (fp32 / generic family): the
    native elementwise kernel (ops/act.py) on GPU, ATen otherwise."""
    from torchbooster_amd.ops.act import activation

    return activation(y, "relu")


def _split32_ok(x: Tensor, w: Tensor, up: int, reflect: bool) -> bool:
    """csrc/conv.hip conv_fwd_split_k: fp32 as split-bf16 MFMA, C % 64 == K % 64 == 0, zero padding."""
    return (not f32_exact() and x.dtype == torch.float32 and w.dtype == torch.float32 and x.shape[1] % 64 == 0 and w.shape[0] % 64 == 0
            and up == 1 and not reflect and x.numel() % 4 == 0)


def _split_pair(t: Tensor, owner: Optional[Tensor], tag: str):
    """(hi, lo) bf16 pair of an fp32 weight-shaped tensor (channels_last); cached on ``owner``
    while it is frozen (the VGG loss networks of the style-transfer examples)."""
    t = t.contiguous(memory_format=torch.channels_last)
    if owner is None or owner.requires_grad:
        return native().split_bf16(t)
    key = (owner.data_ptr(), owner._version, tuple(owner.shape))
    hit = getattr(owner, "_tb_split_" + tag, None)
    if hit is not None and hit[0] == key:
        return hit[1]
    pair = native().split_bf16(t)
    setattr(owner, "_tb_split_" + tag, (key, pair))
    return pair


def _conv_split32(x: Tensor, w: Tensor, b: Optional[Tensor], stride: int, pad: int, owner=None, tag="w") -> Tensor:
    xh, xl = native().split_bf16(x.contiguous(memory_format=torch.channels_last))
    wh, wl = _split_pair(w, owner, tag)
    return native().conv2d_fwd_split32(xh, xl, wh, wl, b, stride, pad, False)


class _ConvAnyFn(torch.autograd.Function):
    """y = conv2d(pad(upsample(x, up), pad, reflect|zero), w, b, stride) on the generic
    kernels (forward, input gradient via dilated-dy conv + fold, split weight gradient),
    each direction autotuned against MIOpen on the materialised input (whose pad /
    upsample kernels the MIOpen candidate is timed with)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, up, reflect):
        x = x.contiguous(memory_format=torch.channels_last)
        exact = x.dtype == torch.float32 and _sync_f32_mode()
        key = (tuple(x.shape), tuple(w.shape), str(x.dtype) + ("/exact" if exact else ""), stride, pad, up, reflect,
               b is not None)

        def nat():
            return native().conv_any_fwd(x, w, b, stride, pad, up, reflect)

        def mio():
            if up == 1 and not reflect:  # plain zero padding: MIOpen pads itself
                return F.conv2d(x, w, b, stride, pad).contiguous(memory_format=torch.channels_last)
            return F.conv2d(_virtual(x, pad, up, reflect), w, b, stride).contiguous(memory_format=torch.channels_last)

        cands = [("native", nat, 0.0), ("miopen", mio, 0.0)]
        if _virt64_ok(x, w, stride, up):  # the 64-channel implicit GEMM with virtual-input addressing
            cands.insert(0, ("native64", lambda: native().conv2d_fwd_virtual(x, w, b, stride, pad, up, reflect), 0.0))
        if _tinyc_ok(x, w, stride, pad, up, reflect):  # im2col row gathered into the MFMA operand
            cands.insert(0, ("tinyc", lambda: native().conv_tinyc_fwd(x, w, b, stride, pad, reflect, False), 0.0))
        if _narrow_ok(x, w, stride, pad, up, reflect):  # K <= 16: halo tile in LDS, taps read from it
            cands.insert(0, ("narrow", lambda: native().conv_narrow_fwd(x, w, b, pad, up, reflect), 0.0))
        if (pad == 0 and up == 1 and x.shape[2] == w.shape[2] and x.shape[3] == w.shape[3]
                and w.is_contiguous(memory_format=torch.channels_last)):
            cands.append(("gemm", lambda: _window_gemm(x, w, b), 0.0))
        if CG.supported(x, w):
            cands.append(("im2col", lambda: CG.conv_fwd(x, w, b, stride, pad, up, reflect), 0.0))
        if _split32_ok(x, w, up, reflect):  # fp32: split-bf16 passes of the implicit-GEMM MFMA kernel
            cands.insert(0, ("split32", lambda: _conv_split32(x, w, b, stride, pad, w, "w"), 0.0))
        if _narrow32_ok(x, w, stride, pad, up, reflect):  # fp32 RGB head: split-bf16 halo-tile runs
            cands.insert(0, ("narrow32", lambda: native().conv_narrow_fwd_split32(x, w, b, pad, up, reflect), 0.0))
        if _tinyhalo_ok(x, w, stride, pad, up, reflect):  # RGB input, stride 1: LDS halo tile
            cands.insert(0, ("tinyhalo", lambda: native().conv_tinyhalo_fwd(x, w, b, pad, reflect, False), 0.0))
        if _tiny32_ok(x, w, stride, pad, up, reflect):  # fp32 RGB input: split-bf16 im2col gather
            cands.insert(0, ("tiny32", lambda: native().conv_tiny32_fwd(x, w, b, stride, pad, reflect, False), 0.0))
        y = _route("fwd", ("any",) + key, cands)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, up, reflect, b is not None)
        ctx.wparam = w
        ctx.bias_ref = b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, up, reflect, has_bias = ctx.cfg
        if torch.is_grad_enabled():  # create_graph: differentiable ATen recompute
            ins = [t for t, need in ((x, ctx.needs_input_grad[0]), (w, ctx.needs_input_grad[1])) if need]
            b = ctx.bias_ref if has_bias else None
            if b is not None and ctx.needs_input_grad[2]:
                ins.append(b)
            y = F.conv2d(_virtual(x, pad, up, reflect), w, b, stride)
            got = list(torch.autograd.grad(y, ins, dy, create_graph=True, allow_unused=True)) if ins else []
            out = [None] * 7
            for i, need in enumerate((ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                                      has_bias and ctx.needs_input_grad[2])):
                if need:
                    out[i] = got.pop(0)
            return tuple(out)
        with torch.no_grad():
            dy = dy.contiguous(memory_format=torch.channels_last)
            exact = x.dtype == torch.float32 and _sync_f32_mode()
            key = (tuple(x.shape), tuple(w.shape), str(x.dtype) + ("/exact" if exact else ""), stride, pad, up,
                   reflect)
            dx = dw = db = None
            if ctx.needs_input_grad[0]:
                def nat_d():
                    return native().conv_any_dgrad(dy, w, x.shape[2], x.shape[3], stride, pad, up, reflect,
                                                   _dgrad_weight(w, ctx.wparam))

                def mio_d():
                    if up == 1 and not reflect:
                        return _miopen_bwd(dy, x, w, stride, pad, 0)
                    return _miopen_dgrad_virtual(dy, x, w, stride, pad, up, reflect)

                cands = [("native", nat_d, 0.0), ("miopen", mio_d, 0.0)]
                R_, S_ = w.shape[2], w.shape[3]
                if (stride == 1 and up == 1 and not reflect and R_ == S_ and pad <= R_ - 1
                        and _narrow_ok(dy, w.transpose(0, 1), 1, R_ - 1 - pad, 1, False)):
                    # input gradient with <= 16 input channels (RGB input convs): the halo-tile
                    # forward on dy with the flipped, transposed weight
                    cands.insert(0, ("narrow", lambda: native().conv_narrow_fwd(
                        dy, w.flip(2, 3).transpose(0, 1), None, R_ - 1 - pad, 1, False), 0.0))
                if (stride > 1 and up == 1 and not reflect and R_ == S_ and dy.dtype == torch.bfloat16
                        and dy.shape[1] in (32, 64) and x.shape[1] <= 16 and -(-R_ // stride) <= 9
                        and (dy.shape[2] - 1) * stride - 2 * pad + R_ == x.shape[2]
                        and (dy.shape[3] - 1) * stride - 2 * pad + S_ == x.shape[3]):
                    # strided conv with <= 16 input channels (DCGAN discriminator input): its input
                    # gradient is a narrow transposed conv of dy -> stride phases on the halo kernel
                    cands.insert(0, ("narrow", lambda: native().conv_narrow_transpose_fwd(
                        dy, w, None, stride, pad), 0.0))
                if _virt64_ok(x, w, stride, up) and (stride == 1 or native().conv_dgrad_s2_supported(R_, S_, 2)):
                    cands.insert(0, ("native64", lambda: native().conv2d_dgrad_virtual(
                        dy, _flipped(w, ctx.wparam), x.shape[2], x.shape[3], stride, pad, up, reflect), 0.0))
                if up == 1 and not reflect and CG.supported(dy, w):
                    cands.append(("im2col", lambda: CG.conv_dgrad(dy, w, x.shape, stride, pad), 0.0))
                if (stride == 1 and up == 1 and not reflect and R_ == S_ and pad <= R_ - 1
                        and _narrow32_ok(dy, w.transpose(0, 1), 1, R_ - 1 - pad, 1, False)):
                    # fp32 input gradient with <= 16 input channels: split-bf16 halo-tile runs on dy
                    cands.insert(0, ("narrow32", lambda: native().conv_narrow_fwd_split32(
                        dy, w.flip(2, 3).transpose(0, 1), None, R_ - 1 - pad, 1, False), 0.0))
                if (stride == 1 and R_ == S_ and pad <= R_ - 1 and dy.dtype == torch.float32
                        and _split32_ok(dy, w.transpose(0, 1), up, reflect)):
                    # stride-1 fp32 input gradient = the split-bf16 forward on dy with the flipped,
                    # transposed weight (cached split while the weight is frozen)
                    cands.insert(0, ("split32", lambda: _conv_split32(
                        dy, w.flip(2, 3).transpose(0, 1), None, 1, R_ - 1 - pad, ctx.wparam, "wt"), 0.0))
                dx = _route("dgrad", ("any",) + key, cands)
            if ctx.needs_input_grad[1]:
                def nat_w():
                    return native().conv_any_wgrad(dy, x, w.shape[2], w.shape[3], stride, pad, up, reflect)

                def mio_w():
                    if up == 1 and not reflect:
                        return _miopen_bwd(dy, x, w, stride, pad, 1)
                    xv = _virtual(x, pad, up, reflect).contiguous(memory_format=torch.channels_last)
                    return _miopen_bwd(dy, xv, w, stride, 0, 1)

                cands = [("native", nat_w, 0.0), ("miopen", mio_w, 0.0)]
                if _tinyhalo_ok(x, w, stride, pad, up, reflect) and w.shape[0] <= 64:
                    # RGB / grey input conv: dyᵀ . im2col from an LDS halo tile
                    cands.insert(0, ("tinyhalo", lambda: native().conv_tinyhalo_wgrad(
                        dy, x, w.shape[2], w.shape[3], pad, reflect), 0.0))
                if _narrow_ok(x, w, stride, pad, up, reflect):
                    cands.insert(0, ("narrow", lambda: native().conv_narrow_wgrad(
                        dy, x, w.shape[2], w.shape[3], pad, up, reflect), 0.0))
                if _virt_wgrad_ok(x, w, stride, up):
                    cands.insert(0, ("native64", lambda: native().conv2d_wgrad_virtual(
                        dy, x, w.shape[2], w.shape[3], stride, pad, up, reflect), 0.0))
                Cn, Kn, Rn, Sn = x.shape[1], w.shape[0], w.shape[2], w.shape[3]
                if (not exact and x.dtype == torch.float32 and dy.dtype == torch.float32 and Cn in (32, 64)
                        and 1 <= Kn <= 16
                        and Rn <= 9 and Sn <= 9 and stride == 1 and up in (1, 2, 4)
                        and (not reflect or (pad < x.shape[2] * up and pad < x.shape[3] * up))
                        and x.numel() % 4 == 0 and dy.numel() % 4 == 0):
                    # fp32 RGB heads (9x9, <= 16 outputs): split-bf16 runs of the halo-tile kernel
                    cands.insert(0, ("narrow32", lambda: native().conv_narrow_wgrad_split32(
                        dy, x, Rn, Sn, pad, up, reflect).contiguous(memory_format=torch.channels_last), 0.0))
                if (not exact and x.dtype == torch.float32 and dy.dtype == torch.float32 and x.shape[1] % 64 == 0
                        and w.shape[0] % 64 == 0 and up in (1, 2, 4) and x.numel() % 4 == 0):
                    # fp32 (the reference precision): split-bf16 passes of the 64-channel MFMA kernel
                    cands.insert(0, ("split32", lambda: native().conv2d_wgrad_split32(
                        dy, x, w.shape[2], w.shape[3], stride, pad, up, reflect), 0.0))
                if CG.supported(x, w):
                    cands.append(("im2col", lambda: CG.conv_wgrad(dy, x, w.shape, stride, pad, up, reflect), 0.0))
                if up == 1 and not reflect and _tinyin_ok(x, dy, w, stride, pad):
                    # RGB-input 4x4 / 2 conv (DCGAN discriminator input): csrc/conv_tinyin_wgrad.hip
                    cands.insert(0, ("tinyin", lambda: native().conv2d_wgrad_tinyin(x, dy), 0.0))
                dw = _route("wgrad", ("any",) + key, cands)
                if not w.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous()
            if has_bias and ctx.needs_input_grad[2]:
                db = _bias_grad(dy, w.dtype)
            return dx, dw, db, None, None, None, None


def _miopen_dgrad_virtual(dy: Tensor, x: Tensor, w: Tensor, stride: int, pad: int, up: int,
                          reflect: bool) -> Tensor:
    """MIOpen input gradient on the materialised virtual input, folded back with ATen's
    own pad / upsample backward (autograd through _virtual)."""
    xv_shape = _virtual(x[:, :, :1, :1].new_zeros(1, 1, x.shape[2], x.shape[3]), pad, up, reflect).shape[2:]
    xv = torch.empty(x.shape[0], x.shape[1], *xv_shape, dtype=x.dtype, device=x.device,
                     memory_format=torch.channels_last)
    gv = _miopen_bwd(dy, xv, w, stride, 0, 0)
    with torch.enable_grad():
        xr = x.detach().requires_grad_()
        v = _virtual(xr, pad, up, reflect)
        g, = torch.autograd.grad(v, xr, gv)
    return g.contiguous(memory_format=torch.channels_last)


def conv2d_any(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, stride: int = 1, padding: int = 0,
               upsample: int = 1, reflect: bool = False) -> Tensor:
    """``conv2d(pad(upsample_nearest(x, upsample), padding, reflect|zero), w, bias, stride)`` with
    the padding and upsampling folded into the kernel's addressing (GPU), ATen otherwise."""
    if conv_any_supported(x, w, stride, padding):
        return _ConvAnyFn.apply(x, w, bias, int(stride), int(padding), int(upsample), bool(reflect))
    return F.conv2d(_virtual(x, int(padding), int(upsample), bool(reflect)), w, bias, stride)


class Conv2d(torch.nn.Conv2d):
    """``nn.Conv2d`` on the native kernels: the implicit-GEMM kernels for bf16 NHWC
    with C_in / C_out multiples of 64, the generic family (csrc/conv_any.hip) for
    other channel counts, fp32, and ``padding_mode="reflect"``; MIOpen otherwise
    (grouped / dilated convs).  State-dict compatible with ``nn.Conv2d``."""

    def forward(self, x: Tensor, relu: bool = False, fold: Optional[Tuple[int, bool, int]] = None) -> Tensor:
        """``relu``: also apply the ReLU that follows this conv (in the native kernel's
        epilogue when it runs natively) -- see :class:`ConvReLUSequential`.  ``fold =
        (pad, reflect, upsample)``: this call's input is the tensor BEFORE a preceding
        nearest-upsample / (reflection) pad, which run inside the conv's addressing
        (nativize's fold; the conv's own padding is replaced by ``pad``)."""
        if fold is not None:  # (pad, reflect, upsample) folded in by nativize(): one native op
            pad, reflect, up = fold
            y = conv2d_any(x, self.weight, self.bias, _pair(self.stride), pad, up, reflect)
            return _relu(y) if relu else y
        if self.padding_mode == "zeros" and x.is_cuda and native_supported(x, self.weight, self.stride, self.padding,
                                                                          self.dilation, self.groups):
            return conv2d(x, self.weight, self.bias, self.stride, self.padding, self.dilation, self.groups, relu)
        if (self.padding_mode in ("zeros", "reflect") and x.is_cuda
                and conv_any_supported(x, self.weight, self.stride, self.padding, self.dilation, self.groups)):
            y = _ConvAnyFn.apply(x, self.weight, self.bias, _pair(self.stride), _pair(self.padding), 1,
                                 self.padding_mode == "reflect")
            return _relu(y) if relu else y
        y = super().forward(x)
        return _relu(y) if relu else y


class ConvReLUSequential(torch.nn.Sequential):
    """``nn.Sequential`` that runs each ``Conv2d -> ReLU`` pair as one conv with the ReLU in
    its epilogue (torchvision VGG ``features``: 16 such pairs in VGG-19).  Module indices,
    state-dict keys and slicing are those of the plain Sequential; a pair is fused only when
    neither module has hooks (the style examples hook conv outputs, offline.yml
    style_layers 0/5/10/19/28, and ReLU outputs, online.yml layers 3/8/15/22 -- hooked
    modules run unfused, so every hook sees exactly what it would in a plain Sequential)."""

    def forward(self, x: Tensor) -> Tensor:
        mods = list(self._modules.values())
        i = 0
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if (isinstance(m, Conv2d) and type(nxt) is torch.nn.ReLU and not _has_hooks(m)
                    and not _has_hooks(nxt)):
                x = m.forward(x, relu=True)
                i += 2
                continue
            x = m(x)
            i += 1
        return x


def _has_hooks(m: torch.nn.Module) -> bool:
    return bool(m._forward_hooks or m._forward_pre_hooks or m._backward_hooks
                or getattr(m, "_backward_pre_hooks", None))


class PadConv2d(torch.nn.Module):
    """``conv(pad(upsample(x)))`` as ONE native op — what :func:`~torchbooster_amd.nativize`
    turns ``ReflectionPad2d -> Conv2d`` and ``Upsample(nearest) -> ReflectionPad2d -> Conv2d``
    chains into (reference StyleNet ``Conv`` / ``DeconvIN``, online.py:46-48, adain.py:36-38).
    Holds the original conv as ``conv`` (state-dict keys unchanged under it)."""

    def __init__(self, conv: torch.nn.Conv2d, pad: int, reflect: bool, upsample: int = 1) -> None:
        super().__init__()
        self.conv = conv
        self.pad, self.reflect, self.upsample = int(pad), bool(reflect), int(upsample)

    def forward(self, x: Tensor) -> Tensor:
        c = self.conv  # (fused only when the conv itself has no padding)
        return conv2d_any(x, c.weight, c.bias, _pair(c.stride), self.pad, self.upsample, self.reflect)


def conv_transpose_supported(x: Tensor, w: Tensor, stride, padding, output_padding=0, dilation=1, groups=1) -> bool:
    """ConvTranspose2d on the native kernels: x [N, Ci, H, W], w [Ci, Co, R, R] bf16 with
    Ci, Co multiples of 64 (the conv it is the input-gradient of has K = Ci, C = Co)."""
    if _DISABLE or _DISABLE_T or not x.is_cuda or x.dim() != 4 or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if groups != 1 or _pair(dilation) != 1 or _pair(output_padding) != 0 or w.shape[2] != w.shape[3]:
        return False
    s, p, R = _pair(stride), _pair(padding), w.shape[2]
    if s not in (1, 2) or p < 0 or p > R - 1:
        return False
    return x.shape[1] % 64 == 0 and w.shape[1] % 64 == 0 and w.shape[0] == x.shape[1]


class _ConvTFn(torch.autograd.Function):
    """y = conv_transpose2d(x, w): the input gradient of conv2d(·, w, stride, pad)
    evaluated at dY = x, so it runs on the dgrad paths (flipped-weight implicit
    GEMM at stride 1, four output-parity sub-convolutions at stride 2).  Its
    backward is the conv forward (dX) and the conv weight gradient with the
    roles of input and output swapped (dW).  SURVEY.md §2.3.1 K27."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, pad):
        N, _, H, W = x.shape
        R = w.shape[2]
        Ho, Wo = (H - 1) * stride - 2 * pad + R, (W - 1) * stride - 2 * pad + R
        shape_of = torch.empty((N, w.shape[1], Ho, Wo), dtype=x.dtype, device=x.device,
                               memory_format=torch.channels_last)  # output geometry (never read)
        y = _dgrad(x, shape_of, w, stride, pad, None, None, None, w)
        y = y.contiguous(memory_format=torch.channels_last)
        if bias is not None:
            y = y.add_(bias.view(1, -1, 1, 1).to(y.dtype))
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, bias is not None)
        ctx.wparam = w
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, has_bias = ctx.cfg
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _fwd(dy, w, None, stride, pad, False)[0]
        if ctx.needs_input_grad[1]:
            slot = take_slot(ctx.wparam)
            if slot is not None and (slot.dtype != w.dtype or not slot.is_contiguous(memory_format=torch.channels_last)):
                slot = None
            dw = _wgrad(x, dy, w, stride, pad, slot)
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(dy, w.dtype)
        return dx, dw, db, None, None


def conv_transpose2d(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, stride=1, padding=0, output_padding=0,
                     groups=1, dilation=1) -> Tensor:
    if use_native(x) and conv_transpose_supported(x, w, stride, padding, output_padding, dilation, groups):
        x = x.contiguous(memory_format=torch.channels_last)
        w = w.contiguous(memory_format=torch.channels_last)
        return _ConvTFn.apply(x, w, bias, _pair(stride), _pair(padding))
    return F.conv_transpose2d(x, w, bias, stride, padding, output_padding, groups, dilation)


def _tinyin_ok(t: Tensor, g: Tensor, w: Tensor, stride: int, pad: int) -> bool:
    """csrc/conv_tinyin_wgrad.hip: bf16, 3-channel T [N, 3, 2P, 128], 64-channel G [N, 64, P, 64], 4x4 / 2 / pad 1."""
    return (t.dtype == torch.bfloat16 and g.dtype == torch.bfloat16 and t.dim() == 4 and g.dim() == 4
            and t.shape[1] == 3 and g.shape[1] == 64 and g.shape[3] == 64 and t.shape[0] == g.shape[0]
            and t.shape[2] == 2 * g.shape[2] and t.shape[3] == 2 * g.shape[3] and tuple(w.shape[2:]) == (4, 4)
            and stride == 2 and pad == 1 and w.numel() == 64 * 3 * 16)


def conv_transpose_any_supported(x: Tensor, w: Tensor, stride, padding, output_padding=0, dilation=1,
                                 groups=1) -> bool:
    """Transposed convs the generic family takes (any channel counts, bf16 / fp32)."""
    if _DISABLE or _DISABLE_T or not x.is_cuda or x.dim() != 4 or x.dtype not in (torch.bfloat16, torch.float32):
        return False
    if w.dtype != x.dtype or groups != 1 or _pair(dilation) != 1 or _pair(output_padding) != 0:
        return False
    s, p, R = _pair(stride), _pair(padding), w.shape[2]
    return w.shape[2] == w.shape[3] and s >= 1 and 0 <= p <= R - 1 and w.shape[0] == x.shape[1] and use_native(x)


class _ConvTAnyFn(torch.autograd.Function):
    """conv_transpose2d(x, w) = input gradient of conv2d(., w) at dY = x: the generic
    dgrad (dilated conv + fold) forward; backward = the generic forward (dX) and weight
    gradient with the roles of input and output swapped (dW).  Each direction autotuned
    against MIOpen.  (DCGAN edge layers: 64 -> 3 channels, 4x4 / 2.)"""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        x = x.contiguous(memory_format=torch.channels_last)
        N, _, H, W = x.shape
        R = w.shape[2]
        Ho, Wo = (H - 1) * stride - 2 * pad + R, (W - 1) * stride - 2 * pad + R
        key = ("anyT", tuple(x.shape), tuple(w.shape), str(x.dtype), stride, pad)

        def nat():
            y = native().conv_any_dgrad(x, w, Ho, Wo, stride, pad, 1, False, _dgrad_weight(w, w))
            return y if b is None else y.add_(b.view(1, -1, 1, 1).to(y.dtype))

        def mio():
            return F.conv_transpose2d(x, w, b, stride, pad).contiguous(memory_format=torch.channels_last)

        cands = [("native", nat, 0.0), ("miopen", mio, 0.0)]
        if (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.shape[1] in (32, 64)
                and w.shape[1] <= 16 and w.shape[2] == w.shape[3] and -(-R // stride) <= 9):
            # <= 16 output channels: stride phases on the halo-tile kernel (csrc/conv_narrow.hip)
            cands.insert(0, ("narrow", lambda: native().conv_narrow_transpose_fwd(x, w, b, stride, pad), 0.0))
        if CG.supported(x, w):
            cands.append(("im2col", lambda: CG.convT_fwd(x, w, b, stride, pad), 0.0))
        y = _route("fwd", key, cands)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, b is not None)
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, has_bias = ctx.cfg
        dy = dy.contiguous(memory_format=torch.channels_last)
        key = ("anyT", tuple(x.shape), tuple(w.shape), str(x.dtype), stride, pad)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            cands = [("native", lambda: native().conv_any_fwd(dy, w, None, stride, pad, 1, False), 0.0),
                     ("miopen", lambda: F.conv2d(dy, w, None, stride, pad).contiguous(memory_format=torch.channels_last),
                      0.0)]
            if _tinyc_ok(dy, w, stride, pad, 1, False):  # RGB dy (generator head): im2col-gather kernel
                cands.insert(0, ("tinyc", lambda: native().conv_tinyc_fwd(dy, w, None, stride, pad, False, False), 0.0))
            dx = _route("dgrad", key, cands)
        if ctx.needs_input_grad[1]:
            R = w.shape[2]

            def nat_w():
                g = native().conv_any_wgrad(x, dy, R, R, stride, pad, 1, False)
                return g if w.is_contiguous(memory_format=torch.channels_last) else g.contiguous()

            cands = [("native", nat_w, 0.0), ("miopen", lambda: _miopen_bwd(x, dy, w, stride, pad, 1), 0.0)]
            if CG.supported(x, w):
                cands.append(("im2col", lambda: CG.convT_wgrad(x, dy, w.shape, stride, pad), 0.0))
            if _tinyin_ok(dy, x, w, stride, pad):
                # 64 -> RGB 4x4 / 2 transposed conv (DCGAN generator output): the mirrored conv's
                # weight gradient with T = dY, G = x (csrc/conv_tinyin_wgrad.hip)
                cands.insert(0, ("tinyin", lambda: native().conv2d_wgrad_tinyin(dy, x), 0.0))
            dw = _route("wgrad", key, cands)
            if not w.is_contiguous(memory_format=torch.channels_last):
                dw = dw.contiguous()
        if has_bias and ctx.needs_input_grad[2]:
            db = _bias_grad(dy, w.dtype)
        return dx, dw, db, None, None


class ConvTranspose2d(torch.nn.ConvTranspose2d):
    """``nn.ConvTranspose2d`` on the native kernels: the 64-channel dgrad/fwd/wgrad
    kernels (bf16, channels multiples of 64, stride 1 or 2), the generic family
    (csrc/conv_any.hip) for other channel counts and fp32; MIOpen otherwise
    (output padding, groups, dilation).  State-dict compatible with ``nn.ConvTranspose2d``."""

    def forward(self, x: Tensor, output_size=None) -> Tensor:
        if (output_size is None and self.padding_mode == "zeros" and x.is_cuda
                and conv_transpose_supported(x, self.weight, self.stride, self.padding, self.output_padding,
                                             self.dilation, self.groups)):
            return conv_transpose2d(x, self.weight, self.bias, self.stride, self.padding)
        if (output_size is None and self.padding_mode == "zeros" and x.is_cuda
                and conv_transpose_any_supported(x, self.weight, self.stride, self.padding, self.output_padding,
                                                 self.dilation, self.groups)):
            return _ConvTAnyFn.apply(x, self.weight, self.bias, _pair(self.stride), _pair(self.padding))
        return super().forward(x, output_size)
