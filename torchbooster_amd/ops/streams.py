"""Backward side stream: weight gradients run concurrently with the input-gradient chain.

A convolution's backward has two independent products: the input gradient (the critical
path -- the next layer's backward needs it) and the weight gradient (needed only by the
optimizer, or by the bucket all-reduce).  On MI355X a single ResNet-50 conv kernel leaves
most of the chip's issue slots idle -- it is latency-bound at ~2.5 TB/s and ~20 % MFMA
(profiles/r02_*/) -- so issuing every weight gradient on a second HIP stream lets the
hardware interleave its workgroups with the dgrad / BatchNorm kernels of the layers below,
instead of serialising the two on one queue (the reference has no such split: its backward
is PyTorch's single-stream autograd).

Protocol (all device-side; no host synchronisation):

* :func:`fork` — the side stream waits for the current (compute) stream, so the
  gradient's inputs are ready; the caller launches the weight-gradient kernel under
  ``torch.cuda.stream(side)`` and calls ``record_stream(side)`` on the tensors it read so
  the caching allocator does not hand their memory out before the side stream is done.
* the first fork of a backward queues an autograd final callback that makes the caller's
  stream wait for the side stream when ``backward()`` returns: the optimizer, GradScaler
  and clipping see finished gradients.
* the fork is cheapest when the kernel that produced the gradient recorded its own completion:
  a BatchNorm backward arms a pooled event (:func:`arm`) that its final kernel records as its
  stop event (csrc/common.h ``tb_launch_ev``) and tags its output (:func:`tag`); the conv
  backward that receives that very tensor makes the side stream wait for the event instead of
  recording a marker on the compute stream (4.6 -> 0.75 us per fork behind a 26 us kernel,
  profiles/r03_fork).  Any other gradient gets the plain event fork.
* :func:`comm_stream` — the DDP bucket all-reduce is issued from the side stream (after it
  waited for the compute stream), so RCCL is ordered after the weight gradients of its
  bucket without stalling the compute stream.

Only zero-copy gradient slots (ops/_ext.py ``take_slot``) are written on the side stream:
autograd then adopts the slot alias as ``p.grad`` without touching its data, so no
AccumulateGrad add races the kernel.  ``TBAMD_WGRAD_STREAM=0`` disables the split.
"""
from __future__ import annotations

import contextlib
import os
import weakref
from typing import Dict, Optional

import torch

_ENABLED = os.environ.get("TBAMD_WGRAD_STREAM", "1") == "1"
# the fork/join also inside a hipGraph capture (the side stream joins the capture through the
# fork event; the final-callback join closes it before capture ends).  Off by default: a replayed
# graph with those cross-stream event nodes ran at HALF the speed of the same graph captured on one
# stream (DCGAN G+D: 89 vs 177 steps/s; ResNet-50 b256: 8,357 vs 11,542 img/s;
# profiles/r04_dcgan/README.md)
_IN_CAPTURE = os.environ.get("TBAMD_WGRAD_STREAM_CAPTURE", "0") == "1"
_SIDE: Dict[int, torch.cuda.Stream] = {}
_PENDING: Dict[int, bool] = {}
_TAG: Dict[int, tuple] = {}  # device -> (weakref to the tagged tensor, its data_ptr, event id)
_STOP_EVENTS = os.environ.get("TBAMD_STOP_EVENTS", "1") == "1"
FORKS = {"stop_event": 0, "marker": 0}  # how the side stream was ordered (tests, diagnostics)


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


# priority of the side stream: "normal" (default) = a torch pool stream at the caller's priority;
# "low" puts the weight gradients BELOW the caller's stream (torch only creates priorities <= 0:
# the stream is made natively, hipStreamCreateWithPriority, and wrapped as an ExternalStream).
# With the weight gradient at 2 workgroups/CU (csrc/conv_wgrad.hip) normal beats low by 0.6-0.9 %
# on the ResNet-50 step (12,793 vs 12,675 img/s; profiles/r05_wgrad/); the caller's stream is never
# changed either way.
# "auto" (default): normal, except when an RCCL process group already exists as the stream is made.
# RCCL and ProcessGroupNCCL take streams from torch's pool first, and the side pool stream then
# shares a hardware queue with the compute stream (GPU_MAX_HW_QUEUES is 4 per priority class).  The
# queue runs in order, so the weight gradients serialise with the input-gradient chain.  Measured
# with the --ddp bench (1-rank RCCL group), both on one queue per the kernel trace: 11,949 img/s
# against 13,518 without the wrapper.  A low-priority side stream gets a queue of its own class:
# 13,288 (profiles/r06_ddp/queue_ab.txt)
_SIDE_PRIORITY = os.environ.get("TBAMD_SIDE_PRIORITY", "auto")


def _rccl_group() -> bool:
    import torch.distributed as tdist

    try:
        return tdist.is_available() and tdist.is_initialized() and tdist.get_backend() == "nccl"
    except Exception:  # pragma: no cover - a backend query on a half-torn-down group
        return False
SIDE_INFO: Dict[int, tuple] = {}  # device -> (priority used, least, greatest) for diagnostics


def _make_side(idx: int) -> torch.cuda.Stream:
    if _SIDE_PRIORITY == "low" or (_SIDE_PRIORITY == "auto" and _rccl_group()):
        try:
            from torchbooster_amd.ops._ext import native

            h, least, greatest = native().stream_create_priority(idx, 1 << 20)  # clamped to the least
            SIDE_INFO[idx] = (least, least, greatest)
            if least > 0:
                return torch.cuda.ExternalStream(h, device=torch.device("cuda", idx))
        except Exception:  # no native library: a normal-priority pool stream
            pass
    SIDE_INFO.setdefault(idx, (0, None, None))
    return torch.cuda.Stream(device=idx)


def on_process_group_init() -> None:
    """An RCCL group just came up (distributed.py init paths): a side stream made before it, at the
    caller's priority, is dropped once idle, so the next backward makes it again under the "auto" rule."""
    if _SIDE_PRIORITY != "auto" or not _rccl_group():
        return
    for idx in list(_SIDE):
        if SIDE_INFO.get(idx, (0,))[0] == 0 and not _PENDING.get(idx, False):
            _SIDE.pop(idx).synchronize()
            SIDE_INFO.pop(idx, None)


def side_stream(device) -> torch.cuda.Stream:
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        s = _SIDE[idx] = _make_side(idx)
    return s


def usable(t: torch.Tensor) -> bool:
    """The split applies: enabled, a GPU tensor (inside a hipGraph capture only with
    ``TBAMD_WGRAD_STREAM_CAPTURE=1``)."""
    return _ENABLED and t.is_cuda and (_IN_CAPTURE or not torch.cuda.is_current_stream_capturing())


def arm(t: torch.Tensor) -> Optional[int]:
    """Arm a pooled completion event for the next native ``tb_launch_ev`` launch (a gradient
    producer about to run); None when the side stream is not in use for ``t``."""
    if not (_STOP_EVENTS and _ENABLED and t.is_cuda) or torch.cuda.is_current_stream_capturing():
        return None
    from torchbooster_amd.ops._ext import native

    return int(native().stop_event_arm())


def tag(out: torch.Tensor, ev: Optional[int]) -> None:
    """After the producer ran: if a launch recorded the armed event, remember that ``out`` is
    complete once that event is (only while ``out`` is alive: its memory cannot be reused)."""
    if ev is None:
        return
    from torchbooster_amd.ops._ext import native

    if native().stop_event_disarm():
        _TAG[out.device.index] = (weakref.ref(out), out.data_ptr(), ev)


def fork(device, dy: Optional[torch.Tensor] = None) -> torch.cuda.Stream:
    """Order the side stream after the current stream (after ``dy``'s producer only, when it
    recorded a completion event); arrange the join at backward end."""
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    side = side_stream(idx)
    main = torch.cuda.current_stream(idx)
    t = _TAG.pop(idx, None)
    if (t is not None and dy is not None and t[0]() is not None and t[1] == dy.data_ptr()
            and dy.device.index == idx):
        from torchbooster_amd.ops._ext import native

        native().stream_wait_stop_event(side.cuda_stream, t[2])
        FORKS["stop_event"] += 1
    else:
        side.wait_stream(main)
        FORKS["marker"] += 1
    if not _PENDING.get(idx, False):
        _PENDING[idx] = True
        try:
            torch.autograd.Variable._execution_engine.queue_callback(lambda: join(idx))
        except RuntimeError:  # not inside a backward: the caller joins explicitly
            _PENDING[idx] = False
    return side


def join(idx: int) -> None:
    """The current stream waits for the side stream (end of a backward)."""
    if _PENDING.get(idx, False):
        torch.cuda.current_stream(idx).wait_stream(_SIDE[idx])
        _PENDING[idx] = False


def pending(device) -> bool:
    idx = torch.device(device).index
    return _PENDING.get(torch.cuda.current_device() if idx is None else idx, False)


def priority_compute(device=None):
    """Run the enclosed block on the cached high-priority compute stream (alias of
    :func:`step_priority`, kept for callers of earlier rounds)."""
    return step_priority(device)


_HIPRI: Dict[int, torch.cuda.Stream] = {}
_HIPRI_ENABLED = os.environ.get("TBAMD_HIPRI_COMPUTE", "1") == "1"


def hipri_stream(device=None) -> Optional[torch.cuda.Stream]:
    """The cached HIGH-priority compute stream of ``device`` (None when disabled / no GPU)."""
    if not _HIPRI_ENABLED or not torch.cuda.is_available():
        return None
    idx = torch.cuda.current_device() if device is None else torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    hs = _HIPRI.get(idx)
    if hs is None:
        hs = _HIPRI[idx] = torch.cuda.Stream(device=idx, priority=-1)
    return hs


@contextlib.contextmanager
def step_priority(device=None):
    """Run the enclosed block (forward AND backward: autograd runs each backward op on its
    forward op's stream) on the cached HIGH-priority compute stream, then hand back to the
    caller's stream.  Opt-in; the framework's default path gets the same ordering from the
    low-priority side stream instead (:func:`side_stream`).  Scoped, not process-wide: on entry the
    priority stream waits for the caller's current stream (the loss and the forward that made
    it), on exit the caller's stream waits for the priority stream, and the caller's current
    stream is restored -- user code after ``utils.step`` (metrics, eval, checkpointing, data
    copies, a ``torch.cuda.stream`` context of its own) runs where it started and sees finished
    gradients and parameters.  A no-op when disabled (``TBAMD_HIPRI_COMPUTE=0``), inside a hipGraph
    capture (the captured stream must stay the capturing one) or when already on the stream."""
    hs = hipri_stream(device)
    if hs is None or torch.cuda.is_current_stream_capturing():
        yield None
        return
    outer = torch.cuda.current_stream(hs.device)
    if outer.cuda_stream == hs.cuda_stream:
        yield hs
        return
    hs.wait_stream(outer)
    try:
        with torch.cuda.stream(hs):
            yield hs
    finally:
        outer.wait_stream(hs)


def comm_stream(device):
    """Context for issuing a collective over gradients that may still be in flight on the
    side stream: the side stream (ordered after the compute stream), else a no-op."""
    if not pending(device):
        return contextlib.nullcontext()
    side = side_stream(device)
    side.wait_stream(torch.cuda.current_stream(side.device))
    return torch.cuda.stream(side)
