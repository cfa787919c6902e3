"""Shipped hipBLASLt/rocBLAS algorithm table for the plain library GEMMs.

The Linear layers run their GEMMs on hipBLASLt (plain library GEMMs; the fused
and reduction-shaped work is in the native kernels).  hipBLASLt's heuristic pick
is not always its fastest solution for the transformer shapes (measured on
MI355X: ViT-B/16 b128 step 32.1 -> 28.2 ms with the tuned picks,
gpurun_out/r20).  Like the shipped conv routing table
(``conv_routes_gfx950.json``, a find-db), ``gemm_tuned_gfx950.csv`` records the
measured-best solution per (op, transpose, M, N, K, ld) key; PyTorch's
TunableOp layer then dispatches those shapes to the recorded solution and
everything else to the default heuristic.  No tuning happens at run time unless
asked for (``TBAMD_GEMM_TUNE=1`` tunes unseen shapes online and writes them to
``TBAMD_GEMM_TABLE_OUT``).

The table's validator lines pin the PyTorch / HIP / hipBLASLt / rocBLAS versions
and the gfx950 arch; on any other stack PyTorch ignores it.  ``utils.boost(True)``
— the reference's speed switch (cudnn.benchmark, /root/reference/torchbooster/
utils.py:29-45) — turns it on.  ``TBAMD_GEMM_TABLE=none`` disables it.
"""
from __future__ import annotations

import os
import tempfile
from typing import Optional

import torch

__all__ = ["enable_tuned_gemms", "SHIPPED_TABLE"]

SHIPPED_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_tuned_gfx950.csv")
_STATE = {"enabled": False}


def enable_tuned_gemms(path: Optional[str] = None, tune: Optional[bool] = None) -> bool:
    """Route the library GEMMs through the tuned-solution table. Returns True if enabled."""
    if not torch.cuda.is_available():
        return False
    table = path or os.environ.get("TBAMD_GEMM_TABLE") or SHIPPED_TABLE
    if table == "none":
        return False
    tune = os.environ.get("TBAMD_GEMM_TUNE", "0") == "1" if tune is None else tune
    import torch.cuda.tunable as tunable

    if _STATE["enabled"] and not tune:
        return True
    # results of online tuning go to a scratch file, never into the package
    out = os.environ.get("TBAMD_GEMM_TABLE_OUT") or os.path.join(tempfile.gettempdir(), "tbamd_gemm_tuned.csv")
    tunable.set_filename(out, insert_device_ordinal=False)
    tunable.enable(True)
    tunable.tuning_enable(bool(tune))
    tunable.record_untuned_enable(False)
    if os.path.exists(table):
        tunable.read_file(table)
    _STATE["enabled"] = True
    return True
