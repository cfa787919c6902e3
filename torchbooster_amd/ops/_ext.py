"""Loader for the in-tree native library ``torchbooster_amd/_C.so``.

GPU code paths call :func:`native` which raises loudly when the extension is
missing: a GPU run must never silently fall back to ATen.  CPU tensors use the
pure-PyTorch reference implementations (they are what the CPU test-suite and
the gloo plumbing configuration exercise).

Debug switches:

* ``TBAMD_LAUNCH_BLOCKING=1`` — every native op is followed by a device
  synchronise, so an asynchronous kernel failure is reported by the op that
  launched it (the native analogue of ``CUDA_LAUNCH_BLOCKING``);
* ``TBAMD_BOUNDS=1`` — load the bounds-checked build ``_C_bounds.so``
  (``python -m torchbooster_amd._build --bounds``): guarded kernel accesses are
  checked against their tensor extents on the device, redirected instead of
  faulting, and the op raises ``RuntimeError`` naming itself and the violated
  access class (implies launch-blocking).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

import torch

_C = None
_ERR: Optional[BaseException] = None


_BOUND_BITS = {1: "conv input gather", 2: "conv weight load", 4: "conv output store", 8: "gemm operand load",
               16: "gemm output store", 32: "conv_any input gather", 64: "conv_any output store",
               128: "conv wgrad operand load"}


class _Checked:
    """Proxy over the native module: each op is followed by a synchronise (and, in the
    bounds build, a read of the device violation flags) so failures name their op."""

    def __init__(self, mod, bounds: bool) -> None:
        self._mod, self._bounds = mod, bounds
        self._cache = {}

    def __getattr__(self, name):
        f = getattr(self._mod, name)
        if not callable(f) or isinstance(f, type):
            return f
        w = self._cache.get(name)
        if w is None:
            mod, bounds = self._mod, self._bounds

            def w(*a, **k):
                out = f(*a, **k)
                if torch.cuda.is_available() and torch.cuda.is_initialized():
                    try:
                        torch.cuda.synchronize()
                    except RuntimeError as e:
                        raise RuntimeError(f"native op {name} failed on the device: {e}") from e
                    if bounds:
                        v = int(mod.bounds_check())
                        if v:
                            what = ", ".join(d for b, d in _BOUND_BITS.items() if v & b)
                            raise RuntimeError(f"native op {name}: out-of-bounds access ({what}; flags {v:#x})")
                return out

            self._cache[name] = w
        return w


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    bounds = os.environ.get("TBAMD_BOUNDS", "0") == "1"
    try:
        _C = importlib.import_module("torchbooster_amd._C_bounds" if bounds else "torchbooster_amd._C")
        if bounds or os.environ.get("TBAMD_LAUNCH_BLOCKING", "0") == "1":
            _C = _Checked(_C, bounds)
    except BaseException as e:  # ImportError or a bad/stale .so
        _ERR = e
        _C = None
    if _C is not None and os.environ.get("TBAMD_F32_EXACT", "0") == "1":
        _C.conv_any_set_f32_split(False)  # fp32 convs on the exact-f32 MFMA instead of split-bf16
    return _C


def available() -> bool:
    return _load() is not None


def native():
    """Return the native module or raise with build instructions."""
    m = _load()
    if m is None:
        raise RuntimeError(
            "torchbooster_amd native extension (_C.so) is not available "
            f"({_ERR!r}); build it with `python -m torchbooster_amd._build`"
        )
    return m


def use_native(*tensors: torch.Tensor) -> bool:
    """True when the op must run on the HIP path (any tensor on a GPU).

    ``TBAMD_FORCE_REFERENCE=1`` routes GPU tensors through the PyTorch
    reference path; it exists only for A/B comparisons in benchmarks.
    """
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if not on_gpu:
        return False
    if os.environ.get("TBAMD_FORCE_REFERENCE", "0") == "1":
        return False
    native()  # raise if missing
    return True


DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def take_slot(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Zero-copy gradient slot of parameter ``p`` for this backward, or None.

    The native DDP wrapper and the fused optimizers keep every gradient in a
    persistent flat buffer; ``p._tb_slot`` is ``p``'s view of it.  When
    ``p.grad`` is None (after ``zero_grad(set_to_none=True)``) a kernel that
    produces ``p``'s gradient may write it straight into the slot and return
    :func:`slot_alias` of it: autograd's AccumulateGrad then adopts that tensor
    as ``p.grad`` without a copy or an add (it steals grads nobody else
    references), and the DDP hook finds it already bound to its bucket.  When
    ``p.grad`` is defined (gradient accumulation) the kernel must return a
    fresh tensor so autograd adds it.

    A slot is handed out at most ONCE per backward: a parameter used by several
    nodes of one graph (a discriminator applied to real, fake and interpolated
    batches; a weight-tied block) gets its contributions summed by autograd's
    input buffer BEFORE AccumulateGrad runs, so a second writer of the same
    slot would overwrite the first one's data under that sum.  The first
    caller takes the slot and marks it; later callers in the same backward get
    None (fresh tensors; autograd then sums out of place and the DDP hook /
    optimizer grad store copy the sum into the slot).  The mark is cleared by a
    post-accumulate-grad hook (once every contribution has been summed) and by
    every ``zero_grad`` path (:func:`release_slot`)."""
    if p is None or p.grad is not None:
        return None
    s = getattr(p, "_tb_slot", None)
    if s is None or getattr(p, "_tb_slot_taken", False):
        return None
    if not getattr(p, "_tb_slot_hooked", False):
        p.register_post_accumulate_grad_hook(release_slot)
        p._tb_slot_hooked = True
    p._tb_slot_taken = True
    return s


def slot_in_use(p: Optional[torch.Tensor]) -> bool:
    """True when ``p``'s slot was already handed out in this backward (``p`` is used by
    several nodes): the caller's fresh gradient will be summed by autograd with the slot
    alias, so any side-stream writer of that slot must be joined first."""
    return p is not None and p.grad is None and getattr(p, "_tb_slot_taken", False)


def release_slot(p: torch.Tensor) -> None:
    """Make ``p``'s gradient slot available to the next backward."""
    p._tb_slot_taken = False


def slot_alias(slot: torch.Tensor) -> torch.Tensor:
    """A new tensor object aliasing ``slot`` (refcount 1, so autograd adopts it)."""
    return slot.as_strided(slot.shape, slot.stride(), slot.storage_offset())


# Parameters rewritten in place by a native kernel (the fused optimizers) keep their
# autograd version counter; caches of values derived from parameters (the flipped
# conv weights of ops/conv.py) key on this generation as well.
_PARAM_GEN = [0]


def bump_param_generation() -> None:
    _PARAM_GEN[0] += 1


def param_generation() -> int:
    return _PARAM_GEN[0]


# Work derived from parameters that is best done right after an optimizer update, on the compute
# stream behind it (ops/conv.py: the flipped dgrad weights of every trainable conv), instead of at
# first use inside the next backward -- there the host-side refresh left the GPU idle (~0.17 ms
# per ResNet-50 step between the first BN backward and the first dgrad, profiles/r04_open).
_UPDATE_HOOKS: list = []


def register_param_update_hook(fn) -> None:
    if fn not in _UPDATE_HOOKS:
        _UPDATE_HOOKS.append(fn)


def run_param_update_hooks() -> None:
    for fn in _UPDATE_HOOKS:
        fn()
