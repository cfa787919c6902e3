"""One routing decision for every rank of a job.

The conv router (ops/conv.py ``_route``) and the GEMM tile tuner (ops/gemm.py ``_tuned``) pick a
kernel per shape by timing the candidates on the first call.  Timed on each rank separately, two
ranks of one data-parallel job can pick different kernels for the same layer (box-to-box timing
spread is up to 25 %, profiles/r02_convstudy): the job then runs at the pace of its slowest pick
and the ranks' numerics differ by kernel.  Here rank 0 is authoritative: it times and publishes
its decision in the process group's key-value store; every other rank waits for that key (the
ranks run the same shapes in the same order) and takes it.  A rank that meets a shape rank 0 never
sees (an uneven last batch) stops waiting after ``TBAMD_TUNE_AGREE_TIMEOUT`` seconds and times it
itself, so a shape seen by one rank only cannot hang the job.  The wait has two stages so that it
scales with what rank 0 is doing: rank 0 marks a key as *started* before it times the candidates
(a first-use MIOpen find can take many seconds); a rank waits ``TBAMD_TUNE_AGREE_TIMEOUT`` for that
mark, and once it is there, up to ``TBAMD_TUNE_AGREE_TIMING_TIMEOUT`` for the decision itself.
Every fallback to a local decision is logged (the ranks may then run different kernels).

Reference: the reference leaves kernel choice to cuDNN's per-process heuristics
(``torch.backends.cudnn.benchmark``, /root/reference/torchbooster/utils.py:30-42).
"""
from __future__ import annotations

import datetime
import json
import logging
import os
from typing import Any, Optional

import torch.distributed as tdist

_TIMEOUT_S = float(os.environ.get("TBAMD_TUNE_AGREE_TIMEOUT", "30"))
_TIMING_TIMEOUT_S = float(os.environ.get("TBAMD_TUNE_AGREE_TIMING_TIMEOUT", "600"))
FALLBACKS = []  # keys this rank decided for itself after a timeout (diagnostics, tests)
_ENABLED = os.environ.get("TBAMD_TUNE_AGREE", "1") == "1"


def _store():
    if not _ENABLED or not tdist.is_available() or not tdist.is_initialized():
        return None
    if tdist.get_world_size() <= 1:
        return None
    try:
        return tdist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001 - a process group without a store: decide locally
        return None


def _name(kind: str, key: Any) -> str:
    return f"tbamd/tune/{kind}/{key!r}"


def shared(kind: str, key: Any) -> Optional[Any]:
    """Rank 0's decision for ``key`` (None on rank 0, on a single process, or after the timeout).
    On rank 0 this marks ``key`` as started: it is about to time it and publish the result."""
    st = _store()
    if st is None:
        return None
    k = _name(kind, key)
    if tdist.get_rank() == 0:
        try:
            st.set(k + "/started", "1")
        except Exception:  # noqa: BLE001 - the other ranks then fall back after the short wait
            pass
        return None
    stage = "start"
    try:
        st.wait([k + "/started"], datetime.timedelta(seconds=_TIMEOUT_S))
        stage = "decision"
        st.wait([k], datetime.timedelta(seconds=_TIMING_TIMEOUT_S))
        return json.loads(st.get(k).decode())
    except Exception:  # noqa: BLE001 - timeout: this rank decides for itself
        FALLBACKS.append((kind, key, stage))
        logging.warning("tune-agree: rank %d decides %s %r itself (no rank-0 %s within %.0f s); "
                        "ranks may run different kernels for this shape", tdist.get_rank(), kind, key,
                        stage, _TIMEOUT_S if stage == "start" else _TIMING_TIMEOUT_S)
        return None


def publish(kind: str, key: Any, value: Any) -> None:
    """Rank 0 publishes ``value`` (JSON-serialisable) as the decision for ``key``."""
    st = _store()
    if st is None or tdist.get_rank() != 0:
        return
    try:
        st.set(_name(kind, key), json.dumps(value))
        st.set(_name(kind, key) + "/started", "1")  # (a decision published without a prior shared())
    except Exception:  # noqa: BLE001 - the other ranks fall back to their own timing
        pass
