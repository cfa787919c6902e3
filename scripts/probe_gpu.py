"""GPU probe: native kernel numerics vs PyTorch + ResNet-50 step timing (stock vs native).

Usage: python scripts/probe_gpu.py [--batch 256] [--steps 10] [--only ours|stock]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def check_kernels():
    from torchbooster_amd.ops import _ext
    from torchbooster_amd.ops.norm import batch_norm_act
    from torchbooster_amd.ops.loss import cross_entropy_accuracy
    from torchbooster_amd.ops.optim import FusedAdamW

    C = _ext.native()
    print("native loaded from", C.__file__, flush=True)
    dev = "cuda"
    torch.manual_seed(0)
    res = {}
    for (N, Cc, H, W, act, withres, dt) in [(8, 64, 14, 14, "relu", True, torch.bfloat16),
                                           (4, 6, 12, 12, "gelu", False, torch.float32),
                                           (16, 256, 7, 7, "none", False, torch.bfloat16),
                                           (2, 48, 9, 9, "silu", True, torch.float32)]:
        x = (torch.randn(N, Cc, H, W, device=dev) * 2 + 0.5).to(dt).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x) if withres else None
        w = torch.randn(Cc, device=dev).requires_grad_()
        b = torch.randn(Cc, device=dev).requires_grad_()
        rm = torch.zeros(Cc, device=dev); rv = torch.ones(Cc, device=dev)
        rm2 = rm.clone(); rv2 = rv.clone()
        xa = x.detach().clone().requires_grad_()
        ra = r.detach().clone().requires_grad_() if r is not None else None
        y = batch_norm_act(xa, w, b, rm, rv, True, 0.1, 1e-5, ra, act)
        g = torch.randn_like(y)
        y.backward(g)
        xr = x.detach().float().clone().requires_grad_()
        rr = r.detach().float().clone().requires_grad_() if r is not None else None
        wr = w.detach().clone().requires_grad_(); br = b.detach().clone().requires_grad_()
        z = F.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5)
        if rr is not None:
            z = z + rr
        yr = {"relu": F.relu, "gelu": F.gelu, "none": lambda t: t, "silu": F.silu}[act](z)
        yr.backward(g.float())
        errs = {
            "y": (y.float() - yr).abs().max().item(),
            "dx": (xa.grad.float() - xr.grad).abs().max().item() / (xr.grad.abs().max().item() + 1e-6),
            "dw": (w.grad - wr.grad).abs().max().item() / (wr.grad.abs().max().item() + 1e-6),
            "db": (b.grad - br.grad).abs().max().item() / (br.grad.abs().max().item() + 1e-6),
            "rm": (rm - rm2).abs().max().item(),
            "rv": (rv - rv2).abs().max().item(),
        }
        if r is not None:
            errs["dres"] = (ra.grad.float() - rr.grad).abs().max().item() / (rr.grad.abs().max().item() + 1e-6)
        res[f"bn_{N}x{Cc}x{H}x{W}_{act}_{dt}"] = errs
    # cross entropy
    for K, dt in [(10, torch.float32), (1000, torch.bfloat16)]:
        lg = torch.randn(300, K, device=dev).to(dt).requires_grad_()
        lab = torch.randint(0, K, (300,), device=dev)
        loss, acc = cross_entropy_accuracy(lg, lab, 0.1)
        loss.backward()
        lr_ = lg.detach().float().requires_grad_()
        l2 = F.cross_entropy(lr_, lab, label_smoothing=0.1)
        l2.backward()
        a2 = (lr_.argmax(-1) == lab).float().mean()
        res[f"ce_{K}_{dt}"] = {"loss": abs(loss.item() - l2.item()), "acc": abs(acc.item() - a2.item()),
                               "grad": (lg.grad.float() - lr_.grad).abs().max().item()}
    # AdamW
    ps = [torch.randn(s, device=dev) for s in [(1000, 33), (17,), (64, 3, 7, 7)]]
    ps[2] = ps[2].contiguous(memory_format=torch.channels_last)
    pa = [p.clone().requires_grad_() for p in ps]
    pb = [p.clone().requires_grad_() for p in ps]
    oa = FusedAdamW(pa, lr=1e-2, weight_decay=0.1)
    ob = torch.optim.AdamW(pb, lr=1e-2, weight_decay=0.1)
    for it in range(5):
        for a, b_ in zip(pa, pb):
            gg = torch.randn_like(a)
            a.grad = gg.clone(); b_.grad = gg.clone()
        oa.step(clip=1.0)
        torch.nn.utils.clip_grad_norm_(pb, 1.0)
        ob.step()
    res["adamw"] = max((a - b_).abs().max().item() for a, b_ in zip(pa, pb))
    print(json.dumps(res, indent=1), flush=True)
    return res


def make_model(native: bool):
    from torchbooster_amd.models import resnet50
    m = resnet50().cuda().to(memory_format=torch.channels_last)
    return m


def time_resnet(mode: str, batch: int, steps: int, warmup: int):
    from torchbooster_amd.ops.loss import cross_entropy_accuracy
    from torchbooster_amd.ops.optim import FusedAdamW
    torch.manual_seed(0)
    if mode == "stock":
        os.environ["TBAMD_FORCE_REFERENCE"] = "1"
    else:
        os.environ["TBAMD_FORCE_REFERENCE"] = "0"
    model = make_model(mode != "stock")
    x = torch.randn(batch, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda")
    if mode == "stock":
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)

        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = model(x)
                loss = F.cross_entropy(logits, y, label_smoothing=0.1)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
            return loss
    else:
        model = model.to(torch.bfloat16)
        xb = x.to(torch.bfloat16)
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)

        def step():
            opt.zero_grad(set_to_none=True)
            logits = model(xb)
            loss, acc = cross_entropy_accuracy(logits, y, 0.1)
            loss.backward()
            opt.step(clip=1.0)
            return loss
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {"mode": mode, "batch": batch, "ms_per_step": dt * 1e3, "img_s": batch / dt, "loss": loss.item()}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    print(torch.__version__, torch.cuda.get_device_name(0), flush=True)
    if not a.no_check:
        check_kernels()
    for mode in ["ours", "stock"]:
        if a.only and a.only != mode:
            continue
        time_resnet(mode, a.batch, a.steps, a.warmup)
