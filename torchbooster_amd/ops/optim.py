"""Fused multi-tensor optimizers: AdamW (+ EMA, + f32 master weights) and SGD.

Drop-in replacements for the two optimizers ``OptimizerConfig.make`` builds
(/root/reference/torchbooster/config.py:418-438).  One HIP launch updates every
parameter of a (param dtype, grad dtype) group (csrc/optim.hip); gradient
clipping and AMP unscale / inf-skip are folded into the same launch through
device-resident scalars, so ``utils.step`` needs no host synchronisation.
SURVEY.md §2.3.1 K11-K14.

Numerics match ``torch.optim.AdamW`` / ``torch.optim.SGD`` (f32 math).  For
bf16/f16 parameters an f32 master copy is kept in the optimizer state
(``master_param``) and the low-precision parameter is re-materialised from it in
the same kernel.  ``state_dict()`` stays ``torch.optim.AdamW``-shaped:
``{state: {i: {step, exp_avg, exp_avg_sq[, max_exp_avg_sq, master_param]}}, param_groups}``.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch
from torch import Tensor
from torch.optim import Optimizer

from torchbooster_amd.ops._ext import bump_param_generation, DTYPE_CODE, native

CHUNK = 32768  # elements per workgroup (upper bound)
MIN_CHUNK = 2048
TARGET_CHUNKS = 1024  # small tensor sets are split finer so the launch still covers the 256 CUs


def _chunk_size(total: int) -> int:
    c = MIN_CHUNK
    while c < CHUNK and (total + c - 1) // c > TARGET_CHUNKS:
        c *= 2
    return c
ALIGN = 64  # elements; keeps every flat-state view 256-B aligned for f32

# slot order must match csrc/optim.hip
SLOT_P, SLOT_G, SLOT_M, SLOT_V, SLOT_PM, SLOT_EMA, SLOT_VMAX, NSLOTS = 0, 1, 2, 3, 4, 5, 6, 8


def _dense(t: Tensor) -> bool:
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _h2d(a: np.ndarray, device: torch.device) -> Tensor:
    """Host table -> device without a host sync (pinned staging, stream-ordered copy): the
    first step of a GradScaler loop builds its tables inside ``scaler.step``."""
    t = torch.from_numpy(a)
    if device.type != "cuda":
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


class _Table:
    """Device pointer table + chunk table for one launch."""

    def __init__(self, device: torch.device, rows: np.ndarray, numels: List[int]):
        chunks = []
        cs = _chunk_size(sum(numels))
        for t, n in enumerate(numels):
            for s in range(0, n, cs):
                chunks.append((t, s, min(cs, n - s)))
        self.nchunks = len(chunks)
        ch = np.zeros((max(1, self.nchunks), 3), dtype=np.int64)
        if chunks:
            ch[: len(chunks)] = np.asarray(chunks, dtype=np.int64)
        self.chunks = _h2d(ch, device)
        self.table = _h2d(np.ascontiguousarray(rows), device)
        self.partial = torch.empty(max(1, self.nchunks), dtype=torch.float32, device=device)


class _FlatState:
    """Flat f32 buffers (one allocation per state kind) with per-param views."""

    def __init__(self, params: List[Tensor], kinds: Iterable[str], device):
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += _align(p.numel())
        self.total = max(off, ALIGN)
        self.buffers: Dict[str, Tensor] = {}
        for k in kinds:
            self.buffers[k] = torch.zeros(self.total, dtype=torch.float32, device=device)

    def view(self, kind: str, i: int, p: Tensor) -> Tensor:
        # same strides as the parameter (e.g. channels_last conv weights) so the
        # kernel can walk param, grad and state in one linear memory order
        return torch.as_strided(self.buffers[kind], p.shape, p.stride(), self.offsets[i])


class _GradStore:
    """Optimizer-owned persistent gradient storage: one flat buffer per grad
    dtype, every ``p.grad`` a strided view into it.  Grad pointers then stay
    fixed across steps (device tables are built once) and ``zero_grad`` is one
    memset per dtype.  Params whose grads are owned by the native DDP wrapper
    are left alone."""

    def __init__(self, params: List[Tensor]):
        self.params = [p for p in params if getattr(p, "_tb_ddp", None) is None]
        by_dt: Dict[torch.dtype, List[Tensor]] = {}
        for p in self.params:
            by_dt.setdefault(p.dtype, []).append(p)
        self.buffers: Dict[torch.dtype, Tensor] = {}
        self.views: Dict[int, Tensor] = {}
        for dt, ps in by_dt.items():
            total = sum(_align(p.numel()) for p in ps)
            buf = torch.zeros(max(total, ALIGN), dtype=dt, device=ps[0].device)
            off = 0
            for p in ps:
                v = torch.as_strided(buf, p.shape, p.stride(), off)
                self.views[id(p)] = v
                p._tb_slot = v  # zero-copy gradient slot (ops/_ext.py take_slot)
                off += _align(p.numel())
            self.buffers[dt] = buf

    def bind(self) -> None:
        for p in self.params:
            v = self.views[id(p)]
            g = p.grad
            if g is None or (g.data_ptr() == v.data_ptr() and g.stride() == v.stride()):
                continue
            v.copy_(g)
            p.grad = v

    def zero(self, set_to_none: bool = False) -> None:
        if set_to_none:  # kernels write the next grads straight into the slots
            for p in self.params:
                p.grad = None
                p._tb_slot_taken = False
            return
        for b in self.buffers.values():
            b.zero_()
        for p in self.params:
            p.grad = self.views[id(p)]


class _FusedBase(Optimizer):
    """Shared machinery: groups params by (param dtype, grad dtype) and keeps
    flat state + device tables cached across steps."""

    _step_supports_amp_scaling = True
    _state_kinds: Tuple[str, ...] = ()

    def __init__(self, params, defaults, master_weights: bool = True):
        super().__init__(params, defaults)
        self.master_weights = master_weights
        self._cache: Dict[Tuple, Any] = {}
        self._flat: Dict[int, _FlatState] = {}
        self._gstore: Optional[_GradStore] = None
        for g in self.param_groups:
            g.setdefault("step", 0)

    # ---------------------------------------------------------------- state
    def _kinds_for(self, group, p: Tensor) -> List[str]:
        kinds = list(self._state_kinds)
        if group.get("amsgrad", False):
            kinds.append("max_exp_avg_sq")
        return kinds

    def _init_group_state(self, gi: int, group) -> _FlatState:
        fs = self._flat.get(gi)
        if fs is not None:
            return fs
        params = group["params"]
        device = params[0].device
        kinds = set()
        for p in params:
            kinds.update(self._kinds_for(group, p))
        need_master = self.master_weights and any(p.dtype != torch.float32 for p in params)
        if need_master:
            kinds.add("master_param")
        if getattr(self, "ema_decay", None) is not None:
            kinds.add("ema")
        fs = _FlatState(params, sorted(kinds), device)
        for i, p in enumerate(params):
            st = self.state[p]
            for k in fs.buffers:
                v = fs.view(k, i, p)
                if k == "master_param":
                    if p.dtype == torch.float32:
                        continue
                    old = st.get(k)
                    v.copy_(old if old is not None else p.detach().float())
                elif k == "ema":
                    old = st.get(k)
                    v.copy_(old if old is not None else p.detach().float())
                else:
                    old = st.get(k)
                    if old is not None:
                        v.copy_(old)
                st[k] = v
        self._flat[gi] = fs
        return fs

    def _table_for(self, gi: int, group, fs: _FlatState, idxs: List[int], pdt, gdt) -> _Table:
        params = group["params"]
        key = (gi, pdt, gdt) + tuple((params[i].data_ptr(), params[i].grad.data_ptr()) for i in idxs)
        tab = self._cache.get((gi, pdt, gdt))
        if tab is not None and tab[0] == key:
            return tab[1]
        rows = np.zeros((len(idxs), NSLOTS), dtype=np.int64)
        for r, i in enumerate(idxs):
            p = params[i]
            st = self.state[p]
            rows[r, SLOT_G] = p.grad.data_ptr()
            rows[r, SLOT_PM] = p.data_ptr()
            if "master_param" in st and p.dtype != torch.float32:
                rows[r, SLOT_P] = st["master_param"].data_ptr()
            else:
                rows[r, SLOT_P] = p.data_ptr()
            for k, slot in (("exp_avg", SLOT_M), ("momentum_buffer", SLOT_M), ("exp_avg_sq", SLOT_V),
                            ("ema", SLOT_EMA), ("max_exp_avg_sq", SLOT_VMAX)):
                if k in st and isinstance(st[k], Tensor):
                    rows[r, slot] = st[k].data_ptr()
        t = _Table(params[idxs[0]].device, rows, [params[i].numel() for i in idxs])
        self._cache[(gi, pdt, gdt)] = (key, t)
        return t

    def _partition(self, group) -> Dict[Tuple[torch.dtype, torch.dtype], List[int]]:
        parts: Dict[Tuple[torch.dtype, torch.dtype], List[int]] = {}
        for i, p in enumerate(group["params"]):
            if p.grad is None:
                continue
            if p.grad.is_sparse:
                raise RuntimeError(f"{type(self).__name__} does not support sparse gradients")
            if not _dense(p) or p.grad.stride() != p.stride():
                raise RuntimeError(f"{type(self).__name__} needs dense params with grads of the same layout")
            parts.setdefault((p.dtype, p.grad.dtype), []).append(i)
        return parts

    # ------------------------------------------------------ hipGraph replay
    def _hyper_values(self, group) -> List[float]:
        return [float(group["lr"])]

    def _hyper(self, gi: int, group) -> Optional[Tensor]:
        """Device scalars of group ``gi`` while a graph is being captured (None otherwise)."""
        if not torch.cuda.is_current_stream_capturing():
            return None
        hp = getattr(self, "_hyper_dev", None)
        if hp is None or gi not in hp:
            raise RuntimeError(f"{type(self).__name__}: call graph_prepare() before capturing a step")
        return hp[gi]

    def graph_prepare(self) -> None:
        """Advance the step counters and upload the step-dependent scalars (lr,
        bias corrections) of every group into the device buffers a captured
        step reads (utils.GraphedStep calls this before each replay and once
        before capture).  The staging goes through a small ring of pinned host
        buffers per group, each reused only after the copy that last read it
        completed (an event): a fresh pinned tensor per call goes to the pinned
        allocator, a host-side allocation on every replay whenever the GPU still
        holds the previous copies."""
        if not hasattr(self, "_hyper_dev"):
            self._hyper_dev: Dict[int, Tensor] = {}
            self._hyper_ring: Dict[int, list] = {}
            self._hyper_tick = 0
        dev = None
        for g in self.param_groups:
            for p in g["params"]:
                dev = p.device
                break
        slot = self._hyper_tick % 4
        self._hyper_tick += 1
        for gi, group in enumerate(self.param_groups):
            self._host_step(gi)
            group["step"] += 1
            vals = self._hyper_values(group)
            ring = self._hyper_ring.get(gi)
            if ring is None or ring[0][0].numel() != len(vals):
                pin = dev is not None and dev.type == "cuda"
                ring = self._hyper_ring[gi] = [
                    [torch.empty(len(vals), dtype=torch.float32, pin_memory=pin), None] for _ in range(4)]
            host, ev = ring[slot]
            if ev is not None:
                ev.synchronize()  # (normally long complete: that copy ran at the start of a replay 4 steps ago)
            host.copy_(torch.tensor(vals, dtype=torch.float32))
            buf = self._hyper_dev.get(gi)
            if buf is None or buf.numel() != len(vals):
                buf = self._hyper_dev[gi] = torch.empty(len(vals), dtype=torch.float32, device=dev)
            buf.copy_(host, non_blocking=True)
            if dev is not None and dev.type == "cuda":
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
                ring[slot][1] = ev

    def _device_step_hyper(self, gi: int, group, found_inf: Tensor) -> Tensor:
        """Loss-scaled (fp16) eager step without a host sync: the group's step counter lives
        on the device and advances by ``1 - found_inf``, and the step-dependent scalars
        (lr, bias corrections) are computed there from it; the kernel itself returns early
        on ``found_inf`` (csrc/optim.hip), so a skipped step changes nothing -- torch's
        semantics, with the host counter synced back only when it is read (state_dict)."""
        if not hasattr(self, "_step_dev"):
            self._step_dev: Dict[int, Tensor] = {}
        sd = self._step_dev.get(gi)
        if sd is None:
            sd = self._step_dev[gi] = torch.full((1,), float(group["step"]), dtype=torch.float64,
                                                 device=found_inf.device)
        sd.add_(1.0 - (found_inf.double() != 0).double())
        b1, b2 = group["betas"]
        lr = torch.full_like(sd, float(group["lr"]))  # (a fill kernel: no host-to-device copy)
        return torch.cat([lr, 1.0 - torch.pow(float(b1), sd), (1.0 - torch.pow(float(b2), sd)).sqrt()]).float()

    def _sync_device_steps(self) -> None:
        for gi, sd in getattr(self, "_step_dev", {}).items():
            self.param_groups[gi]["step"] = int(round(float(sd.item())))

    def _host_step(self, gi: int) -> None:
        """The host counter is about to advance (an unscaled eager step, a captured step's
        graph_prepare, the CPU reference path): fold the device counter back in and drop it,
        so there is ONE source of truth and a later loss-scaled step reseeds from the host
        value (a stale device counter would give wrong Adam bias corrections)."""
        sd = getattr(self, "_step_dev", {}).pop(gi, None)
        if sd is not None:
            self.param_groups[gi]["step"] = int(round(float(sd.item())))

    def _skip_for_inf(self, found_inf: Optional[Tensor]) -> bool:
        """GradScaler found a non-finite grad: skip the whole step, step counter
        included (torch semantics; the CPU reference path does the same).  Eager
        steps read the flag on the host — one sync, only under fp16 loss
        scaling, as torch's own non-fused GradScaler path does.  A captured step
        keeps the in-kernel skip (csrc/optim.hip returns early on found_inf)."""
        if found_inf is None or torch.cuda.is_current_stream_capturing():
            return False
        return float(found_inf.sum()) != 0.0

    # ------------------------------------------------------------- clipping
    def _amp_scalars(self):
        gs = getattr(self, "grad_scale", None)
        fi = getattr(self, "found_inf", None)
        inv = None
        if gs is not None:
            inv = gs.double().reciprocal().float().reshape(1)
        if fi is not None:
            fi = fi.float().reshape(1)
        return inv, fi

    def clip_grad_norm_(self, max_norm: float, inv_scale: Optional[Tensor] = None) -> Tensor:
        """Global L2 norm over every grad this optimizer owns; returns a device
        tensor ``[norm, coef, nonfinite]`` (coef = min(1, max_norm / (norm + 1e-6)))."""
        C = native()
        parts_all = []
        for gi, group in enumerate(self.param_groups):
            fs = self._init_group_state(gi, group)
            for (pdt, gdt), idxs in self._partition(group).items():
                parts_all.append((gdt, self._table_for(gi, group, fs, idxs, pdt, gdt)))
        if not parts_all:
            return None
        if len(parts_all) == 1:
            gdt, t = parts_all[0]
            return C.grad_norm_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[gdt], float(max_norm), inv_scale,
                                  t.partial)
        # several dtype groups: one native pass per group into one partial array, one finalize
        return C.grad_norm_multi([t.chunks for _, t in parts_all], [t.nchunks for _, t in parts_all],
                                 [t.table for _, t in parts_all], [DTYPE_CODE[g] for g, _ in parts_all],
                                 float(max_norm), inv_scale)

    # ------------------------------------------------------- CPU reference
    def _bind_grads(self) -> None:
        if self._gstore is None:
            self._gstore = _GradStore([p for g in self.param_groups for p in g["params"]])
        self._gstore.bind()

    def _on_gpu(self) -> bool:
        for g in self.param_groups:
            for p in g["params"]:
                return p.is_cuda
        return False

    def _ref_grads(self, clip: Optional[float]):
        """Unscaled, clipped f32 grads (reference path)."""
        inv_scale, found_inf = self._amp_scalars()
        if found_inf is not None and float(found_inf.sum()) != 0.0:
            return None
        grads = {}
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    gr = p.grad.detach().float()
                    if inv_scale is not None:
                        gr = gr * inv_scale.to(gr.device)
                    grads[p] = gr
        if clip is not None and grads:
            nrm = torch.norm(torch.stack([torch.norm(x) for x in grads.values()]))
            coef = torch.clamp(clip / (nrm + 1e-6), max=1.0)
            self.last_grad_norm = nrm
            grads = {p: x * coef for p, x in grads.items()}
        return grads

    def _reference_step(self, clip):
        grads = self._ref_grads(clip)
        if grads is None:
            return
        for gi, group in enumerate(self.param_groups):
            if not any(p in grads for p in group["params"]):
                continue
            fs = self._init_group_state(gi, group)
            self._host_step(gi)
            group["step"] += 1
            for p in group["params"]:
                if p not in grads:
                    continue
                st = self.state[p]
                master = st.get("master_param") if p.dtype != torch.float32 else None
                w = master if master is not None else p.detach().float()
                self._ref_update(group, st, w, grads[p])
                if "ema" in st:
                    st["ema"].mul_(self.ema_decay).add_(w, alpha=1 - self.ema_decay)
                p.detach().copy_(w)

    # ------------------------------------------------------------ interface
    def zero_grad(self, set_to_none: bool = True) -> None:
        """Grads living in persistent buffers (native DDP buckets, the
        optimizer's grad store) are unbound with ``set_to_none`` — their slots
        stay, so the next backward writes into them without copies — or
        zeroed in place (one memset per buffer); others follow torch semantics."""
        from torchbooster_amd.parallel import ddp as _ddp

        if set_to_none:
            # steady state: one pass over a cached plan (the classification below costs ~0.1 ms of
            # host time per ResNet-50 step, right where the GPU waits for the backward to start)
            key = (_ddp.WRAP_GEN[0], id(self._gstore), tuple(len(g["params"]) for g in self.param_groups),
                   id(self.param_groups[0]["params"]) if self.param_groups else 0)
            plan = getattr(self, "_zg_plan", None)
            if plan is not None and plan[0] == key and not any(w() is None for w, _ in plan[1]):
                for w, ps in plan[1]:
                    w().zero_grad_buckets(ps, True)
                for p in plan[2]:
                    p.grad = None
                    p._tb_slot_taken = False
                for p in plan[3]:
                    p.grad = None
                return
        params = [p for g in self.param_groups for p in g["params"]]
        if set_to_none:
            import weakref

            owners, rest0 = {}, []
            for p in params:
                tag = getattr(p, "_tb_ddp", None)
                w = tag[0]() if tag is not None else None
                if w is None:
                    rest0.append(p)
                else:
                    owners.setdefault(id(w), [weakref.ref(w), []])[1].append(p)
            owned = {id(p) for p in self._gstore.params} if self._gstore is not None else set()
            self._zg_plan = (key, [(w, ps) for w, ps in owners.values()], [p for p in rest0 if id(p) in owned],
                             [p for p in rest0 if id(p) not in owned])
        rest = _ddp.zero_grad_params(params, set_to_none)
        if self._gstore is not None and rest:
            self._gstore.zero(set_to_none)
            owned = {id(p) for p in self._gstore.params}
            rest = [p for p in rest if id(p) not in owned]
        for p in rest:
            if p.grad is None:
                continue
            if set_to_none:
                p.grad = None
            else:
                if p.grad.grad_fn is not None:
                    p.grad.detach_()
                else:
                    p.grad.requires_grad_(False)
                p.grad.zero_()

    def state_dict(self) -> Dict[str, Any]:
        self._sync_device_steps()
        for group in self.param_groups:
            for p in group["params"]:
                if p in self.state and len(self.state[p]) > 0:
                    self.state[p]["step"] = torch.tensor(float(group["step"]))
        sd = super().state_dict()
        return sd

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        raw = state_dict["state"]
        saved_groups = state_dict["param_groups"]
        super().load_state_dict(state_dict)
        self._flat.clear()
        self._cache.clear()
        for group, sg in zip(self.param_groups, saved_groups):
            steps = []
            for p, idx in zip(group["params"], sg["params"]):
                src = raw.get(idx)
                if src is None:
                    continue
                st = self.state[p]
                for k, v in src.items():
                    if isinstance(v, Tensor) and k != "step":
                        st[k] = v.detach().to(device=p.device, dtype=torch.float32).clone()
                if "step" in src:
                    s = src["step"]
                    steps.append(int(s.item() if isinstance(s, Tensor) else s))
            if steps:
                group["step"] = max(steps)
        self._step_dev = {}
        for gi, group in enumerate(self.param_groups):
            if any(len(self.state[p]) for p in group["params"]):
                self._init_group_state(gi, group)


class FusedAdamW(_FusedBase):
    """AdamW with decoupled weight decay (torch.optim.AdamW numerics), one
    launch per dtype group, optional EMA of the (f32) weights."""

    _state_kinds = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, *, ema_decay: Optional[float] = None,
                 master_weights: bool = True):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid betas: {betas}")
        self.ema_decay = ema_decay
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=amsgrad)
        super().__init__(params, defaults, master_weights)

    @torch.no_grad()
    def step(self, closure=None, clip: Optional[float] = None, clip_coef: Optional[Tensor] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not self._on_gpu():
            self._reference_step(clip)
            return loss
        self._bind_grads()
        C = native()
        bump_param_generation()
        inv_scale, found_inf = self._amp_scalars()
        # loss scaling, eager: no host read of found_inf -- the step counter is kept on the
        # device (_device_step_hyper) and the kernel skips the update itself
        dev_steps = found_inf is not None and not torch.cuda.is_current_stream_capturing()
        coef = clip_coef
        if clip is not None and coef is None:
            out = self.clip_grad_norm_(clip, inv_scale)
            coef = None if out is None else out[1:2]
            self.last_grad_norm = None if out is None else out[0]
        for gi, group in enumerate(self.param_groups):
            parts = self._partition(group)
            if not parts:
                continue
            fs = self._init_group_state(gi, group)
            hyper = self._hyper(gi, group)  # captured step: counters advance in graph_prepare()
            if dev_steps:
                hyper = self._device_step_hyper(gi, group, found_inf)
            elif hyper is None:
                self._host_step(gi)
                group["step"] += 1
            step = group["step"]
            b1, b2 = group["betas"]
            bc1 = 1.0 - b1 ** step
            bc2s = math.sqrt(1.0 - b2 ** step)
            for (pdt, gdt), idxs in parts.items():
                t = self._table_for(gi, group, fs, idxs, pdt, gdt)
                master = pdt != torch.float32 and "master_param" in fs.buffers
                C.adamw_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[pdt], DTYPE_CODE[gdt], master,
                           self.ema_decay is not None, bool(group["amsgrad"]), float(group["lr"]), float(b1),
                           float(b2), float(group["eps"]), float(group["weight_decay"]), bc1, bc2s,
                           float(self.ema_decay or 0.0), coef, inv_scale, found_inf, hyper)
        return loss

    def _hyper_values(self, group) -> List[float]:
        b1, b2 = group["betas"]
        step = group["step"]
        return [float(group["lr"]), 1.0 - b1 ** step, math.sqrt(1.0 - b2 ** step)]

    def _ref_update(self, group, st, w, g):
        b1, b2 = group["betas"]
        step = group["step"]
        w.mul_(1 - group["lr"] * group["weight_decay"])
        st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
        st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
        v = st["exp_avg_sq"]
        if group["amsgrad"]:
            torch.maximum(st["max_exp_avg_sq"], v, out=st["max_exp_avg_sq"])
            v = st["max_exp_avg_sq"]
        den = v.sqrt() / math.sqrt(1 - b2 ** step) + group["eps"]
        w.addcdiv_(st["exp_avg"], den, value=-group["lr"] / (1 - b1 ** step))

    def ema_tensor(self, p: Tensor) -> Tensor:
        return self.state[p]["ema"]

    @torch.no_grad()
    def swap_ema(self) -> None:
        """Swap model weights with their EMA (call twice to swap back)."""
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state.get(p, {})
                if "ema" not in st:
                    continue
                tmp = p.detach().float().clone()
                p.copy_(st["ema"])
                if "master_param" in st and p.dtype != torch.float32:
                    st["master_param"].copy_(st["ema"])
                st["ema"].copy_(tmp)


class FusedSGD(_FusedBase):
    """SGD with momentum / dampening / nesterov / coupled weight decay
    (torch.optim.SGD numerics), one launch per dtype group."""

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, *, master_weights: bool = True):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        super().__init__(params, defaults, master_weights)

    def _kinds_for(self, group, p):
        return ["momentum_buffer"] if group["momentum"] != 0 else []

    def _ref_update(self, group, st, w, g):
        d = g + group["weight_decay"] * w
        if group["momentum"] != 0:
            buf = st["momentum_buffer"]
            if group["step"] == 1:
                buf.copy_(d)
            else:
                buf.mul_(group["momentum"]).add_(d, alpha=1 - group["dampening"])
            d = d + group["momentum"] * buf if group["nesterov"] else buf
        w.add_(d, alpha=-group["lr"])

    @torch.no_grad()
    def step(self, closure=None, clip: Optional[float] = None, clip_coef: Optional[Tensor] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not self._on_gpu():
            self._reference_step(clip)
            return loss
        self._bind_grads()
        C = native()
        bump_param_generation()
        inv_scale, found_inf = self._amp_scalars()
        if self._skip_for_inf(found_inf):
            return loss
        coef = clip_coef
        if clip is not None and coef is None:
            out = self.clip_grad_norm_(clip, inv_scale)
            coef = None if out is None else out[1:2]
        for gi, group in enumerate(self.param_groups):
            parts = self._partition(group)
            if not parts:
                continue
            fs = self._init_group_state(gi, group)
            hyper = self._hyper(gi, group)
            self._host_step(gi)
            first = group["step"] == 0
            if hyper is None:
                group["step"] += 1
            elif first:
                raise RuntimeError("FusedSGD: run at least one eager step before capturing a graph")
            for (pdt, gdt), idxs in parts.items():
                t = self._table_for(gi, group, fs, idxs, pdt, gdt)
                master = pdt != torch.float32 and "master_param" in fs.buffers
                C.sgd_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[pdt], DTYPE_CODE[gdt], master,
                         float(group["momentum"]), float(group["dampening"]), bool(group["nesterov"]),
                         float(group["weight_decay"]), float(group["lr"]), first, coef, inv_scale, found_inf,
                         hyper)
        return loss


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm: float) -> Tensor:
    """Fused global-norm clipping for an arbitrary parameter list (device
    result, no host sync).  Mirrors ``torch.nn.utils.clip_grad_norm_``."""
    if isinstance(parameters, Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.tensor(0.0)
    if not params[0].grad.is_cuda:
        return torch.nn.utils.clip_grad_norm_(params, max_norm)
    C = native()
    by_dt: Dict[torch.dtype, List[Tensor]] = {}
    for p in params:
        by_dt.setdefault(p.grad.dtype, []).append(p)
    tabs = []
    for gdt, ps in by_dt.items():
        rows = np.zeros((len(ps), NSLOTS), dtype=np.int64)
        for r, p in enumerate(ps):
            rows[r, SLOT_G] = p.grad.data_ptr()
        tabs.append((gdt, _Table(ps[0].device, rows, [p.numel() for p in ps])))
    if len(tabs) == 1:
        gdt, t = tabs[0]
        out = C.grad_norm_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[gdt], float(max_norm), None, t.partial)
        C.scale_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[gdt], out[1:2])
        return out[0]
    sq = []
    for gdt, t in tabs:
        o = C.grad_norm_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[gdt], 0.0, None, t.partial)
        sq.append(o[0].double() ** 2)
    nrm = torch.stack(sq).sum().sqrt().float()
    coef = torch.clamp(max_norm / (nrm + 1e-6), max=1.0).reshape(1)
    for gdt, t in tabs:
        C.scale_mt(t.chunks, t.nchunks, t.table, DTYPE_CODE[gdt], coef)
    return nrm
