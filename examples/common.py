"""Shared helpers for the examples (not part of the library API).

``max_iters()`` lets the test-suite and the GPU smoke runs cap every example at a
few iterations (``TBAMD_EXAMPLE_MAX_ITERS``); ``model_dtype(conf)`` picks the
compute dtype: bf16 weights + f32 master copy on MI355X when ``env.fp16`` is set
(bf16 has the f32 exponent range, so no loss scaling is needed), f32 otherwise.
"""
import os

import torch


def max_iters(default: int) -> int:
    v = os.environ.get("TBAMD_EXAMPLE_MAX_ITERS")
    return min(default, int(v)) if v else default


def use_gpu(conf) -> bool:
    return conf.env.n_gpu > 0 and torch.cuda.is_available()


def model_dtype(conf) -> torch.dtype:
    return torch.bfloat16 if (conf.env.fp16 and use_gpu(conf)) else torch.float32


def prepare_model(model, conf, channels_last: bool = True):
    """dtype + memory format, then ``env.make`` (device + native DDP)."""
    if use_gpu(conf):
        model = model.cuda()
        if channels_last:
            model = model.to(memory_format=torch.channels_last)
        model = model.to(model_dtype(conf))
    return conf.env.make(model)


def to_input(x, conf, channels_last: bool = True):
    x = conf.env.make(x)
    if use_gpu(conf):
        x = x.to(model_dtype(conf))
        if channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
    return x


def report_sync(*models) -> None:
    """Multi-rank rehearsals (``TBAMD_REPORT_SYNC=1``): every rank's parameters must be identical
    after the run; rank 0 prints the largest |difference| of the per-parameter float64 sums across
    ranks and raises if any rank disagrees."""
    if os.environ.get("TBAMD_REPORT_SYNC") != "1":
        return
    import torch.distributed as tdist

    if not (tdist.is_available() and tdist.is_initialized()):
        return
    sums = torch.tensor([float(p.detach().double().sum()) for m in models for p in m.parameters()],
                        dtype=torch.float64)
    outs = [torch.zeros_like(sums) for _ in range(tdist.get_world_size())]
    tdist.all_gather(outs, sums.to(next(models[0].parameters()).device).contiguous() if sums.numel() else sums)
    dev = max(float((o.cpu() - outs[0].cpu()).abs().max()) for o in outs) if sums.numel() else 0.0
    if tdist.get_rank() == 0:
        print(f"[sync] world {tdist.get_world_size()} params {sums.numel()} max |rank - rank0| of param sums "
              f"{dev:.3e}", flush=True)
    if dev != 0.0:
        raise RuntimeError(f"ranks diverged: max |param-sum difference| {dev}")
