"""Tracing / profiling: roctx ranges, an entered profiler context, phase timers.

The reference's ``utils.boost(False)`` builds ``torch.autograd.profiler``
objects but never enters them (/root/reference/torchbooster/utils.py:43-44),
so it traces nothing.  Here:

* :func:`range` / :func:`mark` — roctx ranges and markers (``libroctx64`` via
  ctypes; shows up in ``rocprofv3 --marker-trace`` timelines).  Off unless
  ``TBAMD_ROCTX=1`` or :func:`enable_roctx` is called, and a no-op when the
  library is missing, so they can stay in hot loops.
* :func:`profile` — a ``torch.profiler`` session over CPU + HIP activity that
  IS entered, exporting a Chrome trace (and a kernel table) on exit.
* :class:`PhaseTimer` — HIP-event timers per named phase (data / fwd / bwd /
  reduce / optim), read once at the end (no per-step host syncs).

``utils.step`` wraps its phases in :func:`range`, so a marker trace of any
training script shows zero_grad / backward / clip / optimizer / scheduler.
"""
from __future__ import annotations

import contextlib
import ctypes
import glob
import json
import os
from typing import Dict, Iterator, List, Optional

import torch

__all__ = ["enable_roctx", "roctx_available", "range", "mark", "profile", "PhaseTimer"]

_LIB = None
_TRIED = False
_ENABLED = os.environ.get("TBAMD_ROCTX", "0") == "1"


def _load():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    cands: List[str] = []
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    cands += sorted(glob.glob(os.path.join(tlib, "libroctx64*.so*")))
    cands += sorted(glob.glob("/opt/rocm/lib/libroctx64.so*"))
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _LIB = lib
            break
        except (OSError, AttributeError):
            continue
    return _LIB


def roctx_available() -> bool:
    return _load() is not None


def enable_roctx(on: bool = True) -> bool:
    """Turn roctx ranges on/off; returns whether they are active."""
    global _ENABLED
    _ENABLED = bool(on) and roctx_available()
    return _ENABLED


@contextlib.contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - mirrors roctx naming
    """``with trace.range("fwd"): ...`` — a roctx range when enabled."""
    lib = _load() if _ENABLED else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load() if _ENABLED else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def profile(out_dir: Optional[str] = None, enabled: bool = True, record_shapes: bool = False,
            with_stack: bool = False, row_limit: int = 30):
    """Entered ``torch.profiler`` session (CPU + HIP kernels).

    On exit writes ``<out_dir>/trace.json`` (Chrome trace) and
    ``<out_dir>/kernels.txt`` (top kernels by device time) when ``out_dir``."""
    if not enabled:
        yield None
        return
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=record_shapes, with_stack=with_stack) as prof:
        yield prof
    if out_dir is not None:
        os.makedirs(out_dir, exist_ok=True)
        prof.export_chrome_trace(os.path.join(out_dir, "trace.json"))
        key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
        try:
            table = prof.key_averages().table(sort_by=key, row_limit=row_limit)
        except Exception:  # older/newer profiler column names
            table = prof.key_averages().table(row_limit=row_limit)
        with open(os.path.join(out_dir, "kernels.txt"), "w") as f:
            f.write(table)


class PhaseTimer:
    """Accumulate per-phase device time with HIP events; read once.

    ``with timer("fwd"): ...`` records start/end events on the current stream;
    :meth:`summary` synchronises once and returns ms per phase (total and per
    call).  On CPU it falls back to wall-clock ``perf_counter``."""

    def __init__(self) -> None:
        self._ev: Dict[str, List] = {}

    @contextlib.contextmanager
    def __call__(self, name: str):
        if torch.cuda.is_available():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            with range(name):
                yield
            e.record()
            self._ev.setdefault(name, []).append((s, e))
        else:
            import time

            t0 = time.perf_counter()
            with range(name):
                yield
            self._ev.setdefault(name, []).append((t0, time.perf_counter()))

    def summary(self) -> Dict[str, Dict[str, float]]:
        out = {}
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        for k, evs in self._ev.items():
            if evs and isinstance(evs[0][0], float):
                tot = sum((b - a) * 1e3 for a, b in evs)
            else:
                tot = sum(a.elapsed_time(b) for a, b in evs)
            out[k] = {"total_ms": tot, "calls": len(evs), "ms_per_call": tot / max(len(evs), 1)}
        return out

    def dump(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.summary(), f, indent=1)
