"""Gram (split-K SYRK) kernel (csrc/gram.hip) vs a plain PyTorch fp32 reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import _ext  # noqa: E402
from torchbooster_amd.ops.gram import gram, gram_ref, native_supported  # noqa: E402

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    _ext.native()


def _err(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("shape", [(1, 64, 64, 64), (2, 128, 20, 20), (1, 256, 33, 17), (2, 512, 8, 8),
                                   (1, 64, 512, 512), (3, 192, 16, 16)])
def test_gram_fwd_bwd(shape):
    torch.manual_seed(sum(shape))
    B, C, H, W = shape
    f = torch.randn(*shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    f.requires_grad_()
    assert native_supported(f)
    scale = 1.0 / (C * H * W)
    g = gram(f, scale)
    assert g.shape == (B, C, C) and g.dtype == torch.float32
    fr = f.detach().float().requires_grad_()
    gr = gram_ref(fr, scale)
    assert _err(g, gr) < 5e-3
    assert torch.equal(g, g.transpose(1, 2))  # mirrored exactly
    dg = torch.randn_like(g)
    g.backward(dg)
    gr.backward(dg)
    assert _err(f.grad, fr.grad) < 2e-2


def test_gram_deterministic():
    f = torch.randn(1, 128, 96, 96, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    a, b = gram(f, 1.0), gram(f, 1.0)
    assert torch.equal(a, b)


def test_style_gram_uses_native(monkeypatch):
    from torchbooster_amd.models import style
    from torchbooster_amd.ops import gram as G

    def boom(*a, **k):
        raise AssertionError("fell back to the PyTorch reference")

    monkeypatch.setattr(G, "gram_ref", boom)
    f = torch.randn(2, 64, 16, 16, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = torch.bmm(f.float().flatten(2), f.float().flatten(2).transpose(1, 2)) / (64 * 256)
    assert _err(style.gram_matrix(f), ref) < 5e-3
    assert _err(style.gram_matrix_flat(f[:1]), ref[0]) < 5e-3
