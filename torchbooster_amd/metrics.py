"""Metrics (reference: /root/reference/torchbooster/metrics.py).

``accuracy`` / ``Accuracy`` / ``RunningAverage`` keep the reference API.
``RunningAverage.update`` also accepts a device tensor: it is accumulated on
the device and only read back when ``.value`` is requested, removing the
per-iteration ``.item()`` host syncs of the reference loops.
"""
from __future__ import annotations

from typing import Union

import torch
from torch import Tensor
from torch.nn import Module

__all__ = ["accuracy", "Accuracy", "RunningAverage", "Throughput"]


def accuracy(logits: Tensor, labels: Tensor, dim: int = -1) -> Tensor:
    """Batch accuracy ``(argmax(logits) == labels).sum() / N`` as a tensor."""
    return (logits.argmax(dim=dim) == labels).sum() / logits.size(0)


class Accuracy(Module):
    def forward(self, logits: Tensor, labels: Tensor, dim: int = -1) -> Tensor:
        return accuracy(logits, labels, dim=dim)


class RunningAverage:
    """Cumulative mean ``old <- (old * t + new) / (t + 1)``."""

    def __init__(self) -> None:
        self.current = 0
        self._value: Union[float, Tensor] = 0.0

    def update(self, value: Union[float, Tensor]) -> None:
        n = self.current + 1
        if isinstance(value, Tensor):
            v = value.detach().float().reshape(())
            old = self._value if isinstance(self._value, Tensor) else torch.full((), float(self._value),
                                                                               device=v.device)
            self._value = old + (v - old) / n  # stays on device, no sync
        else:
            cur = float(self._value.item()) if isinstance(self._value, Tensor) else self._value
            self._value = (cur * self.current + float(value)) / n
        self.current = n

    @property
    def value(self) -> float:
        if isinstance(self._value, Tensor):
            return float(self._value.item())
        return self._value

    @value.setter
    def value(self, v: float) -> None:
        self._value = v


class Throughput:
    """Samples/s meter over explicit ``start``/``stop`` brackets (device-synchronised)."""

    def __init__(self) -> None:
        self.samples = 0
        self.seconds = 0.0
        self._t0 = None

    def start(self) -> None:
        import time

        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._t0 = time.perf_counter()

    def stop(self, samples: int) -> float:
        import time

        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dt = time.perf_counter() - self._t0
        self.samples += samples
        self.seconds += dt
        return samples / dt if dt > 0 else float("inf")

    @property
    def value(self) -> float:
        return self.samples / self.seconds if self.seconds > 0 else 0.0
