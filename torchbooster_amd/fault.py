"""Fault injection for failure-path tests.

``TORCHBOOSTER_FAULT_INJECT=<rank>:<step>[:<kind>]`` makes :func:`maybe_inject`
(called by ``utils.step`` once per optimisation step) fail on global rank
``rank`` at step ``step`` (1-based):

* ``raise`` (default) — raise :class:`InjectedFault` (an ordinary exception:
  ``distributed.launch`` propagates it and tears down the other ranks);
* ``exit`` — ``os._exit(17)`` (a hard crash: no Python cleanup, the process
  group sees a dead peer);
* ``nan`` — returns ``"nan"`` so the caller poisons the loss (exercises the
  AMP found-inf / skip path).

The reference has no failure handling beyond fail-fast ``mp.spawn`` semantics
(/root/reference/torchbooster/distributed.py:153); this keeps fail-fast and
makes it testable.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

__all__ = ["InjectedFault", "maybe_inject", "reset", "parse_spec"]

_STEP = 0


class InjectedFault(RuntimeError):
    pass


def parse_spec(spec: str) -> Optional[Tuple[int, int, str]]:
    if not spec:
        return None
    parts = spec.split(":")
    if len(parts) not in (2, 3):
        raise ValueError(f"TORCHBOOSTER_FAULT_INJECT must be rank:step[:kind], got {spec!r}")
    kind = parts[2] if len(parts) == 3 else "raise"
    if kind not in ("raise", "exit", "nan"):
        raise ValueError(f"unknown fault kind {kind!r}")
    return int(parts[0]), int(parts[1]), kind


def reset() -> None:
    global _STEP
    _STEP = 0


def _rank() -> int:
    try:
        import torch.distributed as tdist

        if tdist.is_available() and tdist.is_initialized():
            return tdist.get_rank()
    except Exception:
        pass
    return int(os.environ.get("RANK", "0"))


def maybe_inject() -> Optional[str]:
    """Advance the step counter; fire the configured fault when it matches."""
    global _STEP
    _STEP += 1
    spec = parse_spec(os.environ.get("TORCHBOOSTER_FAULT_INJECT", ""))
    if spec is None:
        return None
    rank, step, kind = spec
    if rank != _rank() or step != _STEP:
        return None
    if kind == "exit":
        os._exit(17)
    if kind == "nan":
        return "nan"
    raise InjectedFault(f"injected fault on rank {rank} at step {step}")
