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
* :func:`load_checkpoint` / :meth:`SaveCallback.latest` for resume.
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

__all__ = ["BaseCallback", "SaveCallback", "StateDictable", "try_extract_state_dict", "load_checkpoint"]

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


def try_extract_state_dict(value: Any) -> Any:
    """``state_dict()`` of modules / optimizers / schedulers / grad scalers, raw value otherwise."""
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

    def __init__(self, every: int, n_iter: int, root: Path, prefix: str, primary_only: bool = True) -> None:
        super().__init__()
        self.every = every
        self.n_iter = n_iter
        self.root = root
        self.prefix = prefix
        self.primary_only = primary_only

    @property
    def path(self) -> Path:
        n = len(str(self.n_iter))
        return Path(self.root, f"{self.prefix}_{self.current:0{n}d}.pt")

    def update(self, **kwargs) -> None:
        if self.current % self.every != 0:
            return
        if self.primary_only and not dist.is_primary():
            return
        _atomic_save({k: try_extract_state_dict(v) for k, v in kwargs.items()}, self.path)

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


def load_checkpoint(path: Union[str, Path], map_location: Any = "cpu", **targets) -> Dict[str, Any]:
    """Restore ``targets`` (name -> object with ``load_state_dict``) from a
    :class:`SaveCallback` file; returns the raw dict (plain values included).
    Uses ``weights_only=True`` so loading executes nothing from the file."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    for name, obj in targets.items():
        if name not in ckpt:
            continue
        obj = _unwrap(obj)
        if hasattr(obj, "load_state_dict"):
            obj.load_state_dict(ckpt[name])
    return ckpt
