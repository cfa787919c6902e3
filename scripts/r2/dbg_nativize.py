"""Per-parameter gradient error of nativize(stock resnet18) vs fp32, under several variants."""
import copy, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from torch import nn
from tests.test_nativize import resnet18
from torchbooster_amd.nativize import nativize


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def run(tag, mk):
    torch.manual_seed(0)
    ref = resnet18(10).cuda().to(memory_format=torch.channels_last)
    model = mk(copy.deepcopy(ref).to(torch.bfloat16))
    x = torch.randn(32, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    out = model(x.to(torch.bfloat16))
    out.float().square().mean().backward()
    out_ref = ref(x)
    out_ref.square().mean().backward()
    g_ref = dict(ref.named_parameters())
    errs = [(n, rel(p.grad, g_ref[n].grad)) for n, p in model.named_parameters() if p.grad is not None]
    bad = [(n, round(e, 3)) for n, e in errs if e > 0.05]
    print(f"{tag:12s} out {rel(out, out_ref):.4f} worst {max(e for _, e in errs):.3f} bad {bad[:12]}", flush=True)


run("bf16-aten", lambda m: m)
run("leaf-only", lambda m: nativize(m, fuse=False))
run("full", lambda m: nativize(m))
