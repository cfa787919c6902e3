"""Training-step utilities (reference: /root/reference/torchbooster/utils.py).

Same names and signatures: ``boost``, ``seed``, ``freeze``, ``detach``,
``iter_loader``, ``isinstance_namedtuple``, ``to_tensor``,
``stack_dictionaries``, ``step`` and the ``Tensorable``/``Tensored``/``Device``
type aliases.

Behavioural fixes:
* B5: ``seed(value, deterministic=True)`` accepts ``deterministic`` (the
  online/adain examples call it).  Determinism uses ``warn_only`` so ops
  without a deterministic ROCm kernel warn instead of aborting.
* B6: ``step(accumulate=True)`` keeps gradients: the next non-accumulating
  ``step`` for that optimizer skips its pre-backward ``zero_grad``.
* B17: ``to_tensor`` honours ``dtype``.
* ``boost`` only toggles what actually takes effect (MIOpen find/benchmark
  mode, anomaly detection); the reference's profiler objects were never
  entered (no-ops).  Profiling lives in :mod:`torchbooster_amd.utils.profiling`.
* ``step`` routes clipping + AMP unscale into the fused optimizer kernel when
  the optimizer is a :class:`~torchbooster_amd.ops.optim.FusedAdamW` /
  ``FusedSGD`` (no host sync, one launch).
"""
from __future__ import annotations

import contextlib
import logging
import os
import random
from itertools import chain
from typing import Any, Dict, Iterator, List, Tuple, TypeVar, Union

import numpy as np
import torch
from torch import Tensor
from torch.nn import Module
from torch.nn.utils import clip_grad_norm_
from torch.optim import Optimizer
from torch.utils.data import DataLoader

from torchbooster_amd import fault, trace
from torchbooster_amd.scheduler import BaseScheduler

__all__ = ["boost", "seed", "freeze", "frozen", "detach", "iter_loader", "isinstance_namedtuple", "to_tensor",
           "stack_dictionaries", "step", "Tensorable", "Tensored", "Device", "GraphedStep", "graph_step", "nativize"]

_STATE: Dict[str, Any] = {"seed": None, "deterministic": None, "boost": None}


def _capture_state() -> Dict[str, Any]:
    return dict(_STATE)


def _reapply_state(state: Dict[str, Any], rank: int = 0) -> None:
    """Re-apply parent ``seed``/``boost`` calls inside a spawned rank (A.2 B8)."""
    if state.get("seed") is not None:
        seed(state["seed"], deterministic=bool(state.get("deterministic")))
    if state.get("boost") is not None:
        boost(state["boost"])


def boost(enable: bool = True) -> None:
    """Speed mode: MIOpen benchmark (find) mode on, the shipped tuned-GEMM table
    (ops/gemm_tuning.py) on, anomaly detection off.  ``boost(False)`` enables
    anomaly detection (debugging)."""
    if not enable:
        logging.warning("torchbooster.utils.boost(False) was called. This will enable anomaly detection and "
                        "can impact the training performance")
    _STATE["boost"] = enable
    torch.backends.cudnn.benchmark = enable
    torch.autograd.set_detect_anomaly(mode=not enable)
    if enable and torch.cuda.is_available():
        from torchbooster_amd.ops.gemm_tuning import enable_tuned_gemms

        enable_tuned_gemms()


def seed(value: int = 42, deterministic: bool = True) -> None:
    """Seed python / numpy / torch RNGs; optionally request deterministic kernels."""
    _STATE["seed"] = value
    _STATE["deterministic"] = deterministic
    random.seed(value)
    np.random.seed(value % (2 ** 32))
    torch.manual_seed(value)
    if deterministic:
        os.environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"
        torch.use_deterministic_algorithms(True, warn_only=True)
    else:
        torch.use_deterministic_algorithms(False)


def freeze(module: Module) -> Module:
    for p in module.parameters():
        p.requires_grad = False
    return module


@contextlib.contextmanager
def frozen(*modules: Module):
    """Temporarily stop gradients into ``modules``' parameters (restored on exit).

    Graph construction reads ``requires_grad`` at forward time, so a forward run
    inside this block builds no weight-gradient edges for these modules: the
    backward that follows later (outside the block) skips their weight-gradient
    kernels, and a :class:`~torchbooster_amd.parallel.DistributedDataParallel`
    wrapper around them fires no hook and all-reduces nothing.  This is the
    generator step of a GAN: ``with utils.frozen(D): g_loss = crit(D(G(z)))``
    (the reference computes and all-reduces D's full gradient on every G step,
    gan.py:102-113)."""
    ps = [p for m in modules for p in m.parameters() if p.requires_grad]
    for p in ps:
        p.requires_grad_(False)
    try:
        yield
    finally:
        for p in ps:
            p.requires_grad_(True)


def detach(*tensors: Tensor) -> Union[Tensor, Iterator[Tensor]]:
    if len(tensors) == 1:
        return tensors[0].detach()
    return (t.detach() for t in tensors)


def iter_loader(loader: DataLoader) -> Iterator[Tuple[int, Any]]:
    """Infinite ``(epoch, batch)`` iterator; advances ``sampler.set_epoch`` (and the dataset's
    ``set_epoch`` when it has one: per-epoch random augmentation, data/readers.py)."""
    epoch = 0
    sampler = getattr(loader, "sampler", None)
    dataset = getattr(loader, "dataset", None)

    def _set(e):
        for obj in (sampler, dataset):
            if hasattr(obj, "set_epoch"):
                obj.set_epoch(e)

    _set(epoch)
    it = iter(loader)
    while True:
        try:
            yield epoch, next(it)
        except StopIteration:
            epoch += 1
            _set(epoch)
            it = iter(loader)
            yield epoch, next(it)


def isinstance_namedtuple(obj: Any) -> bool:
    return isinstance(obj, tuple) and hasattr(obj, "_asdict") and hasattr(obj, "_fields")


Tensorable = TypeVar("Tensorable", Tuple[Any], List[Any], Dict[str, Any])
Tensored = TypeVar("Tensored", List[Tensor], Dict[str, Tensor])
Device = Union[str, torch.device]


def to_tensor(data: Any, dtype: torch.dtype = torch.float32, device: Device = "cpu") -> Any:
    """Convert lists / dicts / namedtuples of values to tensors (``dtype`` honoured)."""

    def tensor(element):
        return torch.as_tensor(element, dtype=dtype, device=device)

    if isinstance(data, list):
        return tensor(data[0]) if len(data) == 1 else tensor(data)
    if isinstance_namedtuple(data):
        return data.__class__(*[tensor(v) for v in data._asdict().values()])
    if isinstance(data, dict) or hasattr(data, "__dict__"):
        if hasattr(data, "copy"):
            data = data.copy()
        for k, v in data.items():
            data[k] = tensor(v)
        return data
    return data


def stack_dictionaries(data: List[Dict[str, Tensor]], dim: int = 0) -> Dict[str, Tensor]:
    if len(data) == 0:
        return {}
    keys = list(dict(data[0]).keys())
    return {k: torch.stack([d[k] for d in data], dim) for k in keys}


def _is_fused(optimizer: Optimizer) -> bool:
    from torchbooster_amd.ops.optim import _FusedBase

    return isinstance(optimizer, _FusedBase)


def step(loss: Tensor, optimizer: Optimizer, scheduler: BaseScheduler = None, scaler=None, clip: float = None,
         retain_graph: bool = False, accumulate: bool = False) -> None:
    """One optimisation step (reference utils.py:204-252).

    Order: zero_grad (skipped after accumulation steps) -> (scaled) backward ->
    [accumulate: return] -> unscale + clip -> optimizer step -> scheduler step ->
    scaler update.
    """
    scaling = scaler is not None and getattr(scaler, "is_enabled", lambda: True)()
    # (no stream switching here: the caller's current stream is the compute stream; the native
    # backward's weight gradients go to a LOW-priority side stream, ops/streams.py side_stream)
    _step(loss, optimizer, scheduler, scaler, clip, retain_graph, accumulate, scaling)


def _step(loss, optimizer, scheduler, scaler, clip, retain_graph, accumulate, scaling) -> None:
    if not accumulate and fault.maybe_inject() == "nan":
        loss = loss * float("nan")
    if not getattr(optimizer, "_tb_accumulating", False):
        with trace.range("zero_grad"):
            optimizer.zero_grad(set_to_none=True)
    with trace.range("backward"):
        from torchbooster_amd.parallel.ddp import no_sync_all

        # accumulation micro-steps skip the gradient all-reduce (every live native
        # DDP wrapper); the final step's backward reduces the accumulated sum
        with (no_sync_all() if accumulate else contextlib.nullcontext()):
            if scaling:
                scaler.scale(loss).backward(retain_graph=retain_graph)
            else:
                loss.backward(retain_graph=retain_graph)
    if accumulate:
        optimizer._tb_accumulating = True
        return
    optimizer._tb_accumulating = False

    with trace.range("optimizer"):
        if _is_fused(optimizer):
            kw = {"clip": clip} if clip is not None else {}
            if scaling:
                scaler.step(optimizer, **kw)
            else:
                optimizer.step(**kw)
            if loss.is_cuda and not torch.cuda.is_current_stream_capturing():
                # (the next backward's flipped conv weights, queued now; inside a GraphedStep capture
                # the captured dgrads flip their weights themselves, so the hooks are not recorded)
                from torchbooster_amd.ops._ext import run_param_update_hooks

                run_param_update_hooks()
        else:
            if clip is not None:
                if scaling:
                    scaler.unscale_(optimizer)
                params = chain.from_iterable(g["params"] for g in optimizer.param_groups)
                clip_grad_norm_(params, max_norm=clip)
            if scaling:
                scaler.step(optimizer)
            else:
                optimizer.step()
    if scheduler is not None:
        scheduler.step()
    if scaling:
        scaler.update()


from torchbooster_amd.utils.graph import GraphedStep, graph_step  # noqa: E402
from torchbooster_amd.nativize import nativize  # noqa: E402
