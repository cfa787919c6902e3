"""Host side of the native dense GEMM engine (csrc/gemm.hip).

Three orientations cover every Linear / 1x1-conv product of a training step
(reference: the cuBLAS calls behind ``nn.Linear`` in the GAN / VAE / LeNet /
ResNet heads, /root/reference/examples/img_gen/gan/gan.py:35-48,
examples/img_gen/vae/vae.py:37-55, examples/img_cls/lenet/lenet.py:33-35;
SURVEY.md §2.3.1 K8):

* ``mm_nt(x, w)``   y  = x wᵀ            forward (w = [out, in]), fused bias /
  bias+GELU (pre-activation saved) / residual epilogues;
* ``mm_nn(dy, w)``  dx = dy w            input gradient, w read TRANSPOSED from
  LDS (no wᵀ copy);
* ``mm_tn(dy, x)``  dw = dyᵀ x           weight gradient, both operands read
  transposed, split-K over the rows with an f32 combine pass.

The tile configuration (and split count for ``mm_tn``) is picked per shape by
timing the candidates once on the GPU (like MIOpen's find step); the decisions
are cached per process and can be saved/loaded (``TBAMD_GEMM_TILES``).
"""
from __future__ import annotations

import json
import os
import sys
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from torchbooster_amd.ops import _agree
from torchbooster_amd.ops._ext import native

__all__ = ["mm_nt", "mm_nn", "mm_tn", "supported_nt", "supported_nn", "supported_tn", "tile_table",
           "save_tiles", "load_tiles"]

_AUTOTUNE = os.environ.get("TBAMD_GEMM_AUTOTUNE", "1") != "0"
_TUNE_LOG = os.environ.get("TBAMD_TUNE_LOG", "0") == "1"
_TILE: Dict[Tuple, Tuple[int, int]] = {}  # (kind, P, Q, K) -> (tile, splits)
_NUM_TILES = None  # native().gemm_num_tiles(): tiles 0-15 of csrc/gemm.hip + 16 = the 8-phase 256x256 NT kernel
TILE8 = 16


def _num_tiles() -> int:
    global _NUM_TILES
    if _NUM_TILES is None:
        _NUM_TILES = int(native().gemm_num_tiles())
    return _NUM_TILES
# tile id of the library candidate (hipBLASLt through ATen).  Round 6 made the native engine beat it
# on ViT's N = 768 products (tiles 17 / 18: whole rounds of the 8-phase kernel + a 128 x 128 tail,
# csrc/gemm.hip; profiles/r06_gemm), so the library is no longer a default candidate:
# TBAMD_GEMM_BLAS=1 times it again (kept only where it beats every native tile by the margins below);
# deterministic mode never uses it.
BLAS = -2
_BLAS_CANDIDATE = os.environ.get("TBAMD_GEMM_BLAS", "0") == "1"
_BLAS_MARGIN = float(os.environ.get("TBAMD_GEMM_BLAS_MARGIN", "0.05"))  # relative
_BLAS_MARGIN_MS = float(os.environ.get("TBAMD_GEMM_BLAS_MARGIN_MS", "0.004"))  # absolute
_BLAS_MIN_MS = float(os.environ.get("TBAMD_GEMM_BLAS_MIN_MS", "0.03"))  # not even timed below this
_SPLITS = (1, 2, 4, 8, 16)


def tile_table() -> Dict[Tuple, Tuple[int, int]]:
    return dict(_TILE)


def save_tiles(path: str) -> None:
    rows = [[list(k), list(v)] for k, v in sorted(_TILE.items(), key=str)]
    with open(path, "w") as f:
        json.dump({"device": "gfx950", "tiles": rows}, f)


def load_tiles(path: Optional[str] = None) -> int:
    path = path or os.environ.get("TBAMD_GEMM_TILES") or os.path.join(os.path.dirname(__file__),
                                                                       "gemm_tiles_gfx950.json")
    if path == "none" or not os.path.exists(path):
        return 0
    with open(path) as f:
        data = json.load(f)
    for k, v in data.get("tiles", []):
        _TILE.setdefault(tuple(k), tuple(v))
    return len(data.get("tiles", []))


def _time_ms(fn: Callable[[], object], reps: int = 3) -> float:
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    ms = s.elapsed_time(e) / reps
    if ms < 0.3:  # sub-0.3 ms candidates: a longer window (3 launches are within launch / clock noise)
        n = int(min(40, max(reps, 1.5 / max(ms, 1e-3))))
        s.record()
        for _ in range(n):
            fn()
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / n
    return ms


def _tuned(key: Tuple, run: Callable[[int, int], Tensor], split_k: bool, blas: bool = True,
           extra_splits: Tuple[int, ...] = (), extra_tiles: Tuple[int, ...] = ()) -> Tensor:
    """Run ``run(tile, splits)`` with the tuned configuration for ``key`` (``blas=False``:
    native tiles only -- the library candidate is not even timed; ``extra_splits``: split-K
    factors timed besides the powers of two)."""
    blas = blas and _BLAS_CANDIDATE  # (the library is opt-in: TBAMD_GEMM_BLAS=1)
    if blas and torch.are_deterministic_algorithms_enabled():
        blas = False  # deterministic mode: the native tiles only (fixed-order split-K combine)
    cfg = _TILE.get(key)
    if cfg is not None and cfg[0] == BLAS and not blas:
        cfg = None  # a library decision (TBAMD_GEMM_BLAS=1 run) where the library is not allowed now
    if cfg is None:
        if not _AUTOTUNE or torch.cuda.is_current_stream_capturing():
            return run(-1, 0 if split_k else 1)
        best, cfg, log = float("inf"), (-1, 1), []
        shared = _agree.shared("gemm", key)  # rank 0's decision (multi-rank jobs)
        if isinstance(shared, list) and len(shared) == 2:
            cfg = tuple(int(v) for v in shared)
        else:
            blas_ms = float("inf")
            splits = tuple(sorted(set(_SPLITS + tuple(extra_splits)))) if split_k else (1,)
            for t in list(range(_num_tiles())) + list(extra_tiles) + ([BLAS] if (_BLAS_CANDIDATE and blas) else []):
                if t == BLAS and best < _BLAS_MIN_MS:
                    continue  # launch-bound GEMM: the library cannot win by the margin below
                if split_k and TILE8 < t < TRANS:
                    continue  # (tiles 17 / 18 are NT / NN only: the same kernel as 16 for a weight gradient)
                cand = splits if t != BLAS else (1,)
                for s in cand:
                    try:
                        ms = _time_ms(lambda: run(t, s))
                    except RuntimeError:
                        continue
                    log.append(f"t{t}s{s}={ms:.3f}")
                    if t == BLAS:
                        blas_ms = ms
                    elif ms < best:
                        best, cfg = ms, (t, s)
            # native first: the library GEMM is taken only where it is clearly faster (a relative
            # and an absolute margin: on the few-microsecond GEMMs of LeNet / a GAN head the
            # difference is launch noise)
            if blas_ms < best * (1.0 - _BLAS_MARGIN) - _BLAS_MARGIN_MS:
                best, cfg = blas_ms, (BLAS, 1)
            _agree.publish("gemm", key, list(cfg))
        _TILE[key] = cfg
        if _TUNE_LOG:
            print(f"[gemm-tune] {key} -> tile {cfg[0]} splits {cfg[1]} ({best:.3f} ms)", file=sys.stderr, flush=True)
    return run(*cfg)


def _ok(*ts: Tensor) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


# Feature counts that are not multiples of 8 (LeNet's 84 / 10, a 1-logit GAN
# discriminator head) are zero-padded to the next multiple of 8 on the host:
# the kernel moves k in 16-B chunks and stores 4 / 8 outputs per lane.  Those
# layers are tiny, so the pad copies cost nothing measurable.
def supported_nt(x: Tensor, w: Tensor) -> bool:
    return _ok(x, w)


def supported_nn(dy: Tensor, w: Tensor) -> bool:
    return _ok(dy, w)


def supported_tn(dy: Tensor, x: Tensor) -> bool:
    return _ok(dy, x)


def _r8(n: int) -> int:
    return (n + 7) // 8 * 8


def _pad_last(t: Tensor, n: int) -> Tensor:
    return t if t.shape[-1] == n else torch.nn.functional.pad(t, (0, n - t.shape[-1]))


def _pad_first(t: Tensor, n: int) -> Tensor:
    if t.shape[0] == n:
        return t
    return torch.cat([t, t.new_zeros((n - t.shape[0],) + tuple(t.shape[1:]))], 0)


def _rows(t: Tensor) -> Tensor:
    t2 = t.reshape(-1, t.shape[-1])
    if t2.stride(-1) != 1 or t2.stride(0) % 8 != 0 or t2.data_ptr() % 16 != 0:
        t2 = t2.contiguous()
    return t2


def mm_nt(x: Tensor, w: Tensor, bias: Optional[Tensor] = None, gelu: bool = False,
          residual: Optional[Tensor] = None, out: Optional[Tensor] = None, blas: bool = True, relu: bool = False):
    """epi(x wᵀ [+ bias] [+ residual]); ``gelu`` returns (gelu(z), z); ``relu`` applies a ReLU
    in the epilogue.  ``blas=False`` keeps the product on the native kernels whatever the
    tuner would pick."""
    K, Q = x.shape[-1], w.shape[0]
    Kp, Qp = _r8(K), _r8(Q)
    x2 = _rows(_pad_last(x, Kp))
    P = x2.shape[0]
    wp = _pad_first(_pad_last(w, Kp), Qp)
    bp = None if bias is None else _pad_first(bias, Qp)
    if relu:
        assert not gelu and residual is None
        epi = 6 if bias is not None else 7
    elif gelu:
        epi = 2
    elif residual is not None:
        epi = 3 if bias is not None else 4
    else:
        epi = 1 if bias is not None else 0
    r2 = None if residual is None else _pad_last(residual.reshape(P, Q), Qp)
    o = out if Qp == Q else None
    C = native()

    def run(t, s):
        if t == BLAS:
            z = F.linear(x2, wp, bp)
            if r2 is not None:
                z = z.add_(r2)
            if gelu:  # hipBLASLt GEMM + bias epilogue, then the native GELU pass
                return [native().gelu_fwd(z) if z.numel() % 8 == 0 else F.gelu(z), z]
            if relu:
                z = F.relu_(z)
            if o is not None:
                o.copy_(z)
                return [o]
            return [z]
        return C.gemm(x2, wp, False, bias=bp, residual=r2, epi=epi, want_z=gelu, tile=t, out=o,
                      splits=s if t == TILE8 else 1)

    res = _tuned(("nt", P, Qp, Kp) + (("relu",) if relu else ()), run, False, blas)
    shp = tuple(x.shape[:-1]) + (Q,)
    if Qp != Q:
        res = [r[:, :Q].contiguous() for r in res]
        if out is not None:
            out.copy_(res[0])
            res[0] = out
    if gelu:
        return res[0].view(shp), res[1].view(shp)
    return res[0].view(shp)


# tile ids >= TRANS (mm_nn): the NT kernel ``tile - TRANS`` on the cached transposed weight
TRANS = 100


def mm_nn(dy: Tensor, w: Tensor, out: Optional[Tensor] = None, owner: Optional[Tensor] = None) -> Tensor:
    """dy w  (dy [..., out], w [out, in]) -> [..., in].  ``owner``: the Parameter ``w`` is (the storage
    of): its cached transpose (ops/conv.py ``transposed_linear_weight``, refreshed once per optimizer
    step) lets the product run as NT on the row-read 8-phase kernel -- a timed candidate (tiles
    TRANS + 16 .. 18) beside the NN tiles, which read W through the transposing LDS path."""
    K, Q = dy.shape[-1], w.shape[1]
    Kp, Qp = _r8(K), _r8(Q)
    d2 = _rows(_pad_last(dy, Kp))
    P = d2.shape[0]
    wp = _pad_last(_pad_first(w, Kp), Qp)
    o = out if Qp == Q else None
    C = native()
    wt = None
    if owner is not None and Kp == K and Qp == Q:
        from torchbooster_amd.ops.conv import transposed_linear_weight

        wt = transposed_linear_weight(w, owner)

    def run(t, s):
        if t == BLAS:
            return torch.mm(d2, wp, out=o) if o is not None else d2 @ wp
        if t >= TRANS:
            if wt is None:  # (decided with the cached transpose, which this call does not have)
                t -= TRANS
            else:
                return C.gemm(d2, wt, False, tile=t - TRANS, out=o, splits=1)[0]
        return C.gemm(d2, wp, True, tile=t, out=o, splits=s if t == TILE8 else 1)[0]

    extra = tuple(TRANS + t for t in (TILE8, TILE8 + 1, TILE8 + 2)) if wt is not None else ()
    y = _tuned(("nn", P, Qp, Kp), run, False, extra_tiles=extra)
    if Qp != Q:
        y = y[:, :Q].contiguous()
        if out is not None:
            out.copy_(y)
            y = out
    return y.view(tuple(dy.shape[:-1]) + (Q,))


def mm_tn(dy: Tensor, x: Tensor, out: Optional[Tensor] = None) -> Tensor:
    """dyᵀ x summed over every leading row (dy [..., out], x [..., in]) -> [out, in]."""
    P, Q = dy.shape[-1], x.shape[-1]
    Pp, Qp = _r8(P), _r8(Q)
    d2, x2 = _rows(_pad_last(dy, Pp)), _rows(_pad_last(x, Qp))
    M = d2.shape[0]
    o = out if (Pp == P and Qp == Q) else None
    C = native()

    def run(t, s):
        if t == BLAS:
            return torch.mm(d2.t(), x2, out=o) if o is not None else d2.t() @ x2
        return C.gemm(d2, x2, True, tx=True, tile=t, splits=s, out=o)[0]

    # split factors that fill the chip with the 256 x 256 weight-gradient tiles (a 768 x 3072 output
    # is 36 tiles: 4 splits leave 112 of 256 CUs idle, 7 fill 252 of them)
    tiles = -(-Pp // 256) * -(-Qp // 256)
    fill = tuple(f for f in {max(1, 256 // tiles), max(1, 512 // tiles)} if 1 < f <= 64)
    y = _tuned(("tn", Pp, Qp, M), run, True, extra_splits=fill)
    if Pp != P or Qp != Q:
        y = y[:P, :Q].contiguous()
        if out is not None:
            out.copy_(y)
            y = out
    return y


if _AUTOTUNE:
    load_tiles()

if os.environ.get("TBAMD_GEMM_SAVE"):
    # collect this process's decisions for the shipped table (scripts/merge_tiles.py)
    import atexit

    atexit.register(lambda: _TILE and save_tiles(os.environ["TBAMD_GEMM_SAVE"]))
