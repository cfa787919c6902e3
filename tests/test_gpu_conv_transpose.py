"""Native ConvTranspose2d (dgrad-as-forward, csrc/conv.hip) vs a PyTorch fp32 reference.

Shapes are the DCGAN-128 generator's up-sampling layers (models/dcgan.py)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import _ext  # noqa: E402
from torchbooster_amd.ops import conv as nconv  # noqa: E402

DEV = "cuda"


@pytest.fixture(autouse=True)
def _force_native(monkeypatch):
    _ext.native()
    for d in ("fwd", "dgrad", "wgrad"):
        monkeypatch.setitem(nconv._FORCE, d, "native")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N,Ci,Co,H,s,p", [(8, 128, 1024, 1, 1, 0), (8, 1024, 512, 4, 2, 1), (4, 256, 128, 16, 2, 1),
                                           (4, 128, 64, 32, 2, 1), (2, 64, 64, 24, 1, 1), (2, 64, 128, 9, 2, 1)])
@pytest.mark.parametrize("bias", [False, True])
def test_conv_transpose_fwd_bwd(N, Ci, Co, H, s, p, bias):
    torch.manual_seed(N * Ci + Co + H)
    x = torch.randn(N, Ci, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Ci, Co, 4, 4, device=DEV) / (Ci * 4) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Co, device=DEV).to(torch.bfloat16) if bias else None
    assert nconv.conv_transpose_supported(x, w, s, p)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    x.requires_grad_()
    w.requires_grad_()
    if bias:
        b.requires_grad_()
    y = nconv.conv_transpose2d(x, w, b, s, p)
    yr = F.conv_transpose2d(xr, wr, br, s, p)
    assert y.shape == yr.shape and y.dtype == torch.bfloat16
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    if bias:
        assert _rel(b.grad, br.grad) < 1e-2


def test_dcgan_generator_native_matches_miopen(monkeypatch):
    from torchbooster_amd.models import DCGANGenerator

    torch.manual_seed(0)
    G = DCGANGenerator(128, 64).to(DEV).to(memory_format=torch.channels_last).to(torch.bfloat16)
    z = torch.randn(4, 128, device=DEV, dtype=torch.bfloat16)
    y = G(z)
    y.float().square().mean().backward()
    g_nat = [p.grad.clone() for p in G.parameters()]
    G.zero_grad(set_to_none=True)
    monkeypatch.setattr(nconv, "_DISABLE", True)  # every ConvTranspose2d on MIOpen
    y2 = G(z)
    y2.float().square().mean().backward()
    assert _rel(y, y2) < 2e-2
    for a, b in zip(g_nat, [p.grad for p in G.parameters()]):
        assert _rel(a, b) < 5e-2
