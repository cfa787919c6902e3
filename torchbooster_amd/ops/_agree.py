"""One routing decision for every rank of a job.

The conv router (ops/conv.py ``_route``) and the GEMM tile tuner (ops/gemm.py ``_tuned``) pick a
kernel per shape by timing the candidates on the first call.  Timed on each rank separately, two
ranks of one data-parallel job can pick different kernels for the same layer (box-to-box timing
spread is up to 25 %, profiles/r02_convstudy): the job then runs at the pace of its slowest pick
and the ranks' numerics differ by kernel.  Here rank 0 is authoritative: it times and publishes
its decision in the process group's key-value store; every other rank waits for that key (the
ranks run the same shapes in the same order) and takes it.  A rank that meets a shape rank 0 never
sees (an uneven last batch) stops waiting after ``TBAMD_TUNE_AGREE_TIMEOUT`` seconds and times it
itself, so a shape seen by one rank only cannot hang the job.

Reference: the reference leaves kernel choice to cuDNN's per-process heuristics
(``torch.backends.cudnn.benchmark``, /root/reference/torchbooster/utils.py:30-42).
"""
from __future__ import annotations

import datetime
import json
import os
from typing import Any, Optional

import torch.distributed as tdist

_TIMEOUT_S = float(os.environ.get("TBAMD_TUNE_AGREE_TIMEOUT", "30"))
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
    """Rank 0's decision for ``key`` (None on rank 0, on a single process, or after the timeout)."""
    st = _store()
    if st is None or tdist.get_rank() == 0:
        return None
    k = _name(kind, key)
    try:
        st.wait([k], datetime.timedelta(seconds=_TIMEOUT_S))
        return json.loads(st.get(k).decode())
    except Exception:  # noqa: BLE001 - timeout: this rank decides for itself
        return None


def publish(kind: str, key: Any, value: Any) -> None:
    """Rank 0 publishes ``value`` (JSON-serialisable) as the decision for ``key``."""
    st = _store()
    if st is None or tdist.get_rank() != 0:
        return
    try:
        st.set(_name(kind, key), json.dumps(value))
    except Exception:  # noqa: BLE001 - the other ranks fall back to their own timing
        pass
