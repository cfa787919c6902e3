"""One-shot all-reduce for small buckets over IPC-mapped peer buffers.

A ring all-reduce of a sub-MiB bucket over the 8-GPU xGMI mesh is latency-bound: 2 (n - 1)
dependent hops.  Here every rank maps every other rank's staging buffer (``hipIpcGetMemHandle`` /
``hipIpcOpenMemHandle``, handles exchanged once through the process group) and ONE kernel per rank
copies its bucket into its own staging buffer, flags it to every peer, waits for the peers' flags,
and sums the n buffers itself in rank order -- one hop over all 7 links at once, and results that
are bitwise identical on every rank (csrc/oneshot.hip).

Reference: the reference reduces every DDP bucket through NCCL (torchbooster/config.py:176-178);
its MLP examples (examples/img_gen/gan/gan.py:31-49, vae/vae.py:37-56) have 0.17-4.3 MiB of gradients.

Requirements: all ranks on one node (IPC), world size <= 8, element count % 8 == 0 and the bucket
within the staging capacity (the DDP wrapper falls back to RCCL otherwise).  The native DDP wrapper
uses it for buckets up to ``TBAMD_ONESHOT_MB`` (default 0 = off until an 8-GPU run validates it).
"""
from __future__ import annotations

import os
import socket
from typing import Optional

import torch
import torch.distributed as tdist

from torchbooster_amd.ops._ext import native

__all__ = ["OneShotAllReduce", "oneshot_threshold_bytes"]


def oneshot_threshold_bytes() -> int:
    return int(float(os.environ.get("TBAMD_ONESHOT_MB", "0")) * 2 ** 20)


class OneShotAllReduce:
    """All ranks of ``process_group`` must construct it together (it exchanges IPC handles)."""

    def __init__(self, process_group=None, capacity_mb: float = 2.0, chunk_kb: int = 64,
                 timeout_s: Optional[float] = None) -> None:
        self.group = process_group
        self.rank = tdist.get_rank(process_group)
        self.world = tdist.get_world_size(process_group)
        hosts = [None] * self.world
        tdist.all_gather_object(hosts, socket.gethostname(), group=process_group)
        if len(set(hosts)) != 1:
            raise RuntimeError("OneShotAllReduce: every rank must be on one node (IPC-mapped buffers)")
        if self.world > 8:
            raise RuntimeError("OneShotAllReduce: at most 8 ranks")
        if timeout_s is None:  # how long a call waits for a slow peer before failing loudly
            timeout_s = float(os.environ.get("TBAMD_ONESHOT_TIMEOUT_S", "600"))
        # every step that can fail on ONE rank (allocation, handle export, mapping the peers) is
        # followed by an exchange of per-rank success flags, so a local failure makes EVERY rank
        # raise together and the caller's fallback (ddp.py) is taken rank-consistently
        self.comm, err = None, ""
        try:
            self.comm = native().OneShotComm(self.rank, self.world, int(capacity_mb * 2 ** 20),
                                             int(chunk_kb) * 1024, float(timeout_s))
            blob = self.comm.handles()
        except Exception as e:  # noqa: BLE001 -- reported collectively below
            blob, err = None, f"{type(e).__name__}: {e}"
        blobs = [None] * self.world
        tdist.all_gather_object(blobs, (err, blob), group=process_group)
        self._agree([e for e, _ in blobs], "setup")
        try:
            self.comm.open([b for _, b in blobs])
            err = ""
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
        # (also the barrier: every rank has mapped every buffer before the first call)
        errs = [None] * self.world
        tdist.all_gather_object(errs, err, group=process_group)
        self._agree(errs, "open")

    def _agree(self, errs, what: str) -> None:
        bad = [(r, e) for r, e in enumerate(errs) if e]
        if bad:
            self.comm = None
            raise RuntimeError(f"OneShotAllReduce: {what} failed on rank(s) " +
                               "; ".join(f"{r}: {e}" for r, e in bad))

    @property
    def capacity(self) -> int:
        return int(self.comm.capacity)

    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.is_contiguous() and t.numel() % 8 == 0
                and t.dtype in (torch.float32, torch.bfloat16, torch.float16)
                and t.numel() * t.element_size() <= self.capacity)

    def all_reduce(self, t: torch.Tensor, average: bool = False, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sum (or mean) of ``t`` over the ranks, in place unless ``out`` is given; ordered on the
        current stream like any kernel (no host synchronisation)."""
        if not self.fits(t):
            raise ValueError("OneShotAllReduce: contiguous f32/bf16/f16 device tensor, numel % 8 == 0, "
                             f"at most {self.capacity} bytes")
        dst = t if out is None else out
        self.comm.allreduce(t, dst, 1.0 / self.world if average else 1.0)
        return dst

    def check(self) -> None:
        """Raise if a call timed out waiting for a peer (its output chunk was poisoned with NaN).
        Reads a host-pinned word the kernel writes: no synchronisation."""
        if self.comm.error():
            raise RuntimeError("OneShotAllReduce: a peer did not arrive within the timeout "
                               "(TBAMD_ONESHOT_TIMEOUT_S; mismatched collective sequence or a stalled rank)")
