"""Training callbacks and checkpointing (reference: /root/reference/torchbooster/callbacks.py).

``SaveCallback(every, n_iter, root, prefix)`` writes
``root/{prefix}_{current:0{len(str(n_iter))}d}.pt`` every ``every`` calls, each
file a ``torch.save`` of ``{kwarg: state_dict-or-value}`` with DDP wrappers
unwrapped (no ``module.`` prefix) — byte-compatible layout with the reference
(callbacks.py:75-129).

Additions:
* duck-typed ``state_dict`` extraction (``torch.amp.GradScaler``, the native
  DDP wrapper, fused optimizers);
* primary-rank-only writes and tmp-file + rename atomicity;
* :func:`load_checkpoint` / :meth:`SaveCallback.latest` for resume;
* exact resume: a ``DataLoader`` / sampler argument is stored as its sampler
  epoch (restored with ``set_epoch``), and with ``save_rng=True`` the file also
  carries an ``rng_state`` entry (Python / NumPy / torch CPU / this rank's GPU
  generator) that :func:`load_checkpoint` puts back (``restore_rng``), so a
  resumed run draws the same shuffles, augmentations and dropout masks as an
  uninterrupted one.  Off by default: the file then holds exactly the
  reference's keys (consumers iterating the dict see nothing extra).
"""
from __future__ import annotations

import os
import re
import tempfile
from pathlib import Path
from typing import Any, Dict, Optional, Union

import torch
from torch.nn import Module
from torch.optim import Optimizer

import torchbooster_amd.distributed as dist
from torchbooster_amd.scheduler import BaseScheduler

__all__ = ["BaseCallback", "SaveCallback", "StateDictable", "try_extract_state_dict", "load_checkpoint",
           "rng_state", "set_rng_state"]

StateDictable = Union[Module, Optimizer, BaseScheduler, Any]


class BaseCallback:
    """``__call__`` increments ``current`` then dispatches to ``update``."""

    def __init__(self) -> None:
        super().__init__()
        self.current = 0

    def __call__(self, *args, **kwargs) -> None:
        self.current += 1
        self.update(*args, **kwargs)

    def update(self, *args, **kwargs) -> None:
        raise NotImplementedError("Method 'update' is not implemented.")


def _unwrap(value: Any) -> Any:
    # torch DDP, the native DDP wrapper, torch.compile-style wrappers
    while hasattr(value, "module") and isinstance(value, Module) and isinstance(value.module, Module):
        value = value.module
    return value


RNG_KEY = "rng_state"


def rng_state() -> Dict[str, Any]:
    """Every generator's state in ``weights_only``-loadable types (tensors, ints, tuples)."""
    import random

    import numpy as np

    name, keys, pos, has_gauss, cached = np.random.get_state()
    out = {"python": random.getstate(), "numpy": (name, torch.from_numpy(keys.astype(np.int64)), int(pos),
                                                   int(has_gauss), float(cached)),
           "torch": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        # only THIS rank's device: get_rng_state_all() would create a context on
        # every visible GPU (other ranks' devices) at each save
        out["cuda"] = torch.cuda.get_rng_state(torch.cuda.current_device())
    return out


def set_rng_state(st: Dict[str, Any]) -> None:
    import random

    import numpy as np

    if "python" in st:
        v = st["python"]
        random.setstate((v[0], tuple(v[1]), v[2]))
    if "numpy" in st:
        name, keys, pos, has_gauss, cached = st["numpy"]
        np.random.set_state((name, keys.numpy().astype(np.uint32), pos, has_gauss, cached))
    if "torch" in st:
        torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        cuda = st["cuda"]
        if isinstance(cuda, (list, tuple)):  # files written by round-2 builds: per-device list
            cuda = cuda[min(torch.cuda.current_device(), len(cuda) - 1)] if len(cuda) else None
        if cuda is not None:
            torch.cuda.set_rng_state(cuda, torch.cuda.current_device())


def _sampler_of(value: Any):
    from torch.utils.data import DataLoader

    if isinstance(value, DataLoader):
        value = value.sampler if value.batch_sampler is None else getattr(value.batch_sampler, "sampler",
                                                                             value.sampler)
    return value if hasattr(value, "set_epoch") else None


def try_extract_state_dict(value: Any) -> Any:
    """``state_dict()`` of modules / optimizers / schedulers / grad scalers; a
    DataLoader / sampler with ``set_epoch`` -> ``{"sampler_epoch": epoch}``; raw
    value otherwise."""
    from torch.utils.data import DataLoader, Sampler

    if isinstance(value, (DataLoader, Sampler)):
        smp = _sampler_of(value)
        return {"sampler_epoch": int(getattr(smp, "epoch", 0))} if smp is not None else {}
    value = _unwrap(value)
    if isinstance(value, (Module, Optimizer, BaseScheduler)):
        return value.state_dict()
    sd = getattr(value, "state_dict", None)
    if callable(sd) and not isinstance(value, (dict, torch.Tensor)):
        try:
            return sd()
        except NotImplementedError:
            return value
    return value


def _atomic_save(obj: Dict[str, Any], path: Path) -> None:
    path.parent.mkdir(parents=True, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=f".{path.name}.", dir=str(path.parent))
    os.close(fd)
    try:
        torch.save(obj, tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)


class SaveCallback(BaseCallback):
    """Save a checkpoint every ``every`` calls (see module docstring)."""

    def __init__(self, every: int, n_iter: int, root: Path, prefix: str, primary_only: bool = True,
                 save_rng: bool = False) -> None:
        super().__init__()
        self.every = every
        self.n_iter = n_iter
        self.root = root
        self.prefix = prefix
        self.primary_only = primary_only
        self.save_rng = save_rng

    @property
    def path(self) -> Path:
        n = len(str(self.n_iter))
        return Path(self.root, f"{self.prefix}_{self.current:0{n}d}.pt")

    def update(self, **kwargs) -> None:
        if self.current % self.every != 0:
            return
        if self.primary_only and not dist.is_primary():
            return
        obj = {k: try_extract_state_dict(v) for k, v in kwargs.items()}
        if self.save_rng and RNG_KEY not in obj:
            obj[RNG_KEY] = rng_state()
        _atomic_save(obj, self.path)

    def latest(self) -> Optional[Path]:
        """Most recent checkpoint written with this prefix under root (or None)."""
        pat = re.compile(rf"^{re.escape(self.prefix)}_(\d+)\.pt$")
        best, best_i = None, -1
        root = Path(self.root)
        if not root.exists():
            return None
        for f in root.iterdir():
            m = pat.match(f.name)
            if m and int(m.group(1)) > best_i:
                best, best_i = f, int(m.group(1))
        return best

    def resume(self, **targets) -> Dict[str, Any]:
        """Load the latest checkpoint into ``targets`` and continue numbering after it."""
        p = self.latest()
        if p is None:
            return {}
        out = load_checkpoint(p, **targets)
        m = re.search(r"_(\d+)\.pt$", p.name)
        if m:
            self.current = int(m.group(1))
        return out


def load_checkpoint(path: Union[str, Path], map_location: Any = "cpu", restore_rng: bool = True,
                    **targets) -> Dict[str, Any]:
    """Restore ``targets`` (name -> object with ``load_state_dict``, or a DataLoader /
    sampler whose epoch is set) from a :class:`SaveCallback` file, and the RNG
    state when the file has one; returns the raw dict (plain values included).
    Uses ``weights_only=True`` so loading executes nothing from the file."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    for name, obj in targets.items():
        if name not in ckpt:
            continue
        smp = _sampler_of(obj)
        if smp is not None and isinstance(ckpt[name], dict) and "sampler_epoch" in ckpt[name]:
            smp.set_epoch(int(ckpt[name]["sampler_epoch"]))
            continue
        obj = _unwrap(obj)
        if hasattr(obj, "load_state_dict"):
            obj.load_state_dict(ckpt[name])
    if restore_rng and isinstance(ckpt.get(RNG_KEY), dict):
        set_rng_state(ckpt[RNG_KEY])
    return ckpt
