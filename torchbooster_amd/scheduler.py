"""Learning-rate schedulers (reference: /root/reference/torchbooster/scheduler.py).

``CycleScheduler`` builds up to three phases — warmup (``decay[0]``,
``lr*initial_multiplier -> lr``), plateau (linear, ``lr -> lr``) and anneal
(``decay[1]``, ``lr -> lr*final_multiplier``) — and each ``step()`` writes
``f(from, to, phase_step / n)`` into every param group (scheduler.py:115-172).

Parity notes:
* the curve values are the reference's, including its ``n + 1`` steps per phase
  (t runs 0/n .. n/n) — B3;
* B2 fixed: the plateau phase is ``"lin"`` (the reference's ``"linear"`` key
  raised ``KeyError`` for any plateau > 0);
* B3 fixed: stepping past the last phase holds the final lr instead of raising
  ``IndexError``.
* The schedule is host-side Python; nothing here touches the GPU.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, Tuple

from torch.optim import Optimizer

__all__ = ["BaseScheduler", "CycleScheduler", "anneal_linear", "anneal_cos", "anneal_exp", "anneal_flat",
           "PHASE_2_FUN"]


def anneal_linear(a: float, b: float, t: float) -> float:
    return a + t * (b - a)


def anneal_cos(a: float, b: float, t: float) -> float:
    return b + 0.5 * (a - b) * (1.0 + math.cos(math.pi * t))


def anneal_exp(a: float, b: float, t: float) -> float:
    return a * (b / a) ** t


def anneal_flat(a: float, b: float, t: float) -> float:
    return a


PHASE_2_FUN = {"lin": anneal_linear, "cos": anneal_cos, "exp": anneal_exp, "flat": anneal_flat}
# accept the long spellings too (the reference's plateau used "linear")
_ALIASES = {"linear": "lin", "cosine": "cos", "exponential": "exp", "constant": "flat"}


def _fun(name: str):
    return PHASE_2_FUN[_ALIASES.get(name, name)]


class BaseScheduler:
    """Base class: ``state_dict`` / ``load_state_dict`` / ``step`` must be overridden."""

    def __init__(self, optimizer: Optimizer) -> None:
        self.optimizer = optimizer

    def state_dict(self) -> Dict[str, Any]:
        raise NotImplementedError("Method 'state_dict' not implemented.")

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        raise NotImplementedError("Method 'load_state_dict' not implemented.")

    def step(self) -> float:
        raise NotImplementedError("Method 'step' not implemented.")


class CycleScheduler(BaseScheduler):
    """Warmup / plateau / anneal learning-rate cycle.

    Attributes ``phases`` (list of ``(kind, lr_from, lr_to, n)``), ``phase``,
    ``phase_step`` and ``last_lr`` mirror the reference and form the
    ``state_dict``.
    """

    def __init__(self, optimizer: Optimizer, lr: float, n_iter: int, initial_multiplier: float = 4e-2,
                 final_multiplier: float = 1e-5, warmup: int = 0, plateau: int = 0,
                 decay: Tuple[str, str] = ("cos", "cos")) -> None:
        super().__init__(optimizer)
        warm_kind, anneal_kind = decay
        phases: List[Tuple[str, float, float, int]] = []
        if warmup > 0:
            phases.append((warm_kind, lr * initial_multiplier, lr, warmup))
        if plateau > 0:
            phases.append(("lin", lr, lr, plateau))
        phases.append((anneal_kind, lr, lr * final_multiplier, n_iter - warmup - plateau))
        self.phases = phases
        self.phase = 0
        self.phase_step = 0
        self.last_lr = None

    def state_dict(self) -> Dict[str, Any]:
        return {"phases": self.phases, "phase": self.phase, "phase_step": self.phase_step,
                "last_lr": self.last_lr}

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        self.phases = [tuple(p) for p in state_dict["phases"]]
        self.phase = state_dict["phase"]
        self.phase_step = state_dict["phase_step"]
        self.last_lr = state_dict["last_lr"]

    def __repr__(self) -> str:
        return f"{type(self).__name__}(phases={[p[0].upper() for p in self.phases]})"

    def _value(self) -> float:
        if self.phase >= len(self.phases):
            kind, a, b, n = self.phases[-1]
            return _fun(kind)(a, b, 1.0) if n > 0 else a
        kind, a, b, n = self.phases[self.phase]
        t = self.phase_step / n if n > 0 else 1.0
        return _fun(kind)(a, b, t)

    def step(self) -> float:
        lr = self._value()
        for group in self.optimizer.param_groups:
            group["lr"] = lr
        self.last_lr = lr
        if self.phase < len(self.phases):
            self.phase_step += 1
            if self.phase_step > self.phases[self.phase][3]:
                self.phase += 1
                self.phase_step = 0
        return lr
