"""Whole-training-step hipGraph capture for launch-bound models.

SURVEY.md §7.4 hard part 4: the reference's small-model workloads (LeNet and
the MLP GAN/VAE at batch 256, /root/reference/examples/img_cls/lenet/lenet.py,
/root/reference/examples/img_gen/gan/gan.py:102-113, vae.py) issue a few
hundred tiny kernels per step, so the step time is host launch latency, not
GPU work.  :class:`GraphedStep` records ``fn`` — forward, loss, backward
(``utils.step`` without its scheduler) and the fused optimizer update — once
into a hipGraph and replays it: one launch per step.

What makes the step capturable:

* every native op launches on the current stream and never syncs the host;
* gradients live in persistent slots (the optimizer's grad store), so the
  captured kernels write the same addresses on every replay;
* the fused optimizers read lr and the Adam bias corrections from a device
  buffer while a graph is captured; :meth:`~torchbooster_amd.ops.optim._FusedBase.graph_prepare`
  advances the step counters and uploads them before every replay, so
  LR schedulers keep working (they run on the host, after the replay);
* conv routing is autotuned during the eager warm-up steps, never in capture;
* the warm-up steps run on the capture stream (PyTorch's side-stream warm-up
  rule): autograd's AccumulateGrad nodes remember the stream they were created
  on, and a node created on the default stream and kept alive by the caller
  (e.g. forward-hook outputs from the previous step) would make the captured
  backward synchronise with the default stream, which capture forbids.

Models must route their GEMM/conv work through kernels that are capturable;
the native ops are.  Steps that depend on MIOpen kernels with workspace
allocation (stride-2 conv / transposed-conv backward, e.g. the DCGAN) are not
supported: run those eagerly.

Inputs are copied into static buffers before each replay; outputs (e.g. the
loss) are static tensors overwritten by every replay.  On CPU (or with
``enabled=False``) the step simply runs eagerly, so code written against
:class:`GraphedStep` runs unchanged in the CPU test-suite.
"""
from __future__ import annotations

from typing import Any, Callable, Iterable, Optional, Sequence

import torch
from torch import Tensor

__all__ = ["GraphedStep", "graph_step"]


def _tree_map(fn, x):
    if isinstance(x, Tensor):
        return fn(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_tree_map(fn, v) for v in x)
    if isinstance(x, dict):
        return {k: _tree_map(fn, v) for k, v in x.items()}
    return x


class GraphedStep:
    """``step = GraphedStep(fn, optimizers, schedulers)``; ``out = step(*inputs)``.

    ``fn(*inputs)`` must run one complete training step (zero_grad, forward,
    backward, optimizer step) on the fused optimizers given here and return
    tensors; LR schedulers are stepped by this object after each step.
    The first ``warmup`` calls run eagerly (autotuning, allocator warm-up,
    optimizer state init), then the step is captured and replayed.
    """

    def __init__(self, fn: Callable[..., Any], optimizers: Iterable = (), schedulers: Iterable = (),
                 warmup: int = 3, enabled: Optional[bool] = None) -> None:
        self.fn = fn
        self.optimizers = list(optimizers)
        self.schedulers = list(schedulers)
        self.warmup = max(1, int(warmup))
        self.enabled = enabled
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_in: Optional[Sequence[Tensor]] = None
        self.static_out: Any = None
        self.calls = 0
        self.stream: Optional[torch.cuda.Stream] = None

    def _use_graph(self, inputs: Sequence[Tensor]) -> bool:
        if self.enabled is not None:
            return bool(self.enabled) and torch.cuda.is_available()
        return torch.cuda.is_available() and all(t.is_cuda for t in inputs if isinstance(t, Tensor))

    def _after(self) -> None:
        for s in self.schedulers:
            s.step()

    def __call__(self, *inputs: Tensor) -> Any:
        self.calls += 1
        if not self._use_graph(inputs):
            out = self.fn(*inputs)
            self._after()
            return out
        if self.stream is None:
            self.stream = torch.cuda.Stream()
        if self.calls <= self.warmup:
            main = torch.cuda.current_stream()
            self.stream.wait_stream(main)
            with torch.cuda.stream(self.stream):
                out = self.fn(*inputs)
            main.wait_stream(self.stream)
            self._after()
            return out
        if self.graph is None:
            self._capture(inputs)
        else:
            for s, x in zip(self.static_in, inputs):
                if s.data_ptr() != x.data_ptr():
                    s.copy_(x, non_blocking=True)
        for o in self.optimizers:
            o.graph_prepare()
        self.graph.replay()
        # the replayed optimizer kernels rewrote the parameters without the host seeing it: caches
        # derived from them (ops/conv.py _FlipCache, refreshed by eager dgrads) are stale now
        from torchbooster_amd.ops._ext import bump_param_generation

        bump_param_generation()
        self._after()
        return self.static_out

    def _capture(self, inputs: Sequence[Tensor]) -> None:
        from torchbooster_amd.ops.optim import _FusedBase

        for o in self.optimizers:
            if not isinstance(o, _FusedBase):
                raise TypeError("GraphedStep needs the fused optimizers (torchbooster_amd.ops.optim)")
        self.static_in = [x.clone() for x in inputs]
        torch.cuda.synchronize()
        # device buffers for the step-dependent scalars must exist before capture;
        # graph_prepare() advanced the counters, undo that (the replay re-advances)
        for o in self.optimizers:
            o.graph_prepare()
            for g in o.param_groups:
                g["step"] -= 1
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            self.static_out = self.fn(*self.static_in)
        torch.cuda.synchronize()


def graph_step(fn: Callable[..., Any], optimizers: Iterable = (), schedulers: Iterable = (), warmup: int = 3,
               enabled: Optional[bool] = None) -> GraphedStep:
    """Functional alias of :class:`GraphedStep`."""
    return GraphedStep(fn, optimizers, schedulers, warmup, enabled)
