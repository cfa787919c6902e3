"""BN apply passes on the short-lived-workgroup grid (csrc/norm_bn.hip bn_apply_blocks, 32768 cap) walking
their rows last-written-first (TBAMD_BN_REVERSE; profiles/r06_bnwg/): the grid and the order only change
which workgroup streams which rows, so a ResNet block's
forward output, input gradient and parameter gradients must be BIT-identical to the old 2048-workgroup
layout and to the uncapped grid.  The cap is read once per process (static initialiser), so each
layout runs in its own subprocess on the same inputs.
Reference: BatchNorm2d + ReLU in the img_cls examples (/root/reference/examples/img_cls/resnet/resnet.py:111).
"""
import os
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from torchbooster_amd import models
torch.manual_seed(0)
dev = torch.device("cuda", 0)
m = models.resnet50(num_classes=10).to(dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
x = torch.randn(8, 3, 96, 96, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
x.requires_grad_(True)
out = m(x).float()
(out * torch.linspace(-1, 1, out.numel(), device=dev).view_as(out)).sum().backward()
torch.cuda.synchronize()
res = {"out": out.detach().cpu(), "dx": x.grad.float().cpu()}
for n, p in m.named_parameters():
    res["g." + n] = p.grad.float().cpu()
for n, b in m.named_buffers():
    res["b." + n] = b.float().cpu()
torch.save(res, sys.argv[2])
"""


def _run(wg: str, path: str, rev: str = "1") -> dict:
    # (kernel choices pinned: no first-use timing that could pick different routes per process)
    env = dict(os.environ, TBAMD_BN_APPLY_WG=wg, TBAMD_BN_REVERSE=rev, TBAMD_CONV_AUTOTUNE="0",
               TBAMD_GEMM_AUTOTUNE="0")
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, path], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return torch.load(path, weights_only=True)


def test_bn_apply_grid_is_bitwise_neutral():
    with tempfile.TemporaryDirectory() as d:
        ref = _run("2048", os.path.join(d, "a.pt"), rev="0")
        for wg, rev in (("32768", "1"), ("16384", "1"), ("131072", "1"), ("32768", "0")):
            got = _run(wg, os.path.join(d, f"{wg}_{rev}.pt"), rev)
            assert got.keys() == ref.keys()
            for k in ref:
                assert torch.equal(got[k], ref[k]), (wg, rev, k, (got[k] - ref[k]).abs().max().item())
