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


def test_gram_backward_runs_native_kernels_only():
    """the Gram backward was a torch.bmm (hipBLASLt); now one native
    symmetrisation pass + native GEMMs."""
    from torch.profiler import ProfilerActivity, profile

    f = torch.randn(2, 128, 32, 32, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    f.requires_grad_()
    g = gram(f, 1.0 / (128 * 32 * 32))
    dg = torch.randn_like(g)
    g.backward(dg, retain_graph=True)  # tune outside the profiled region
    f.grad = None
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        g.backward(dg)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert any("gram_sym_k" in n for n in names) and any("gemm" in n for n in names), names
    assert not any(n.startswith("Cijk") or "bmm" in n for n in names), names


@pytest.mark.parametrize("shape", [(1, 64, 32, 32), (3, 32, 16, 16), (2, 3, 20, 20)])
def test_gram_f32_native_matches_fp32(shape):
    """The reference's f32 precision: exact-f32 MFMA Gram + backward, no hipBLASLt."""
    from torch.profiler import ProfilerActivity, profile

    torch.manual_seed(sum(shape))
    B, C, H, W = shape
    f = torch.randn(*shape, device=DEV).contiguous(memory_format=torch.channels_last).requires_grad_()
    scale = 1.0 / (C * H * W)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        g = gram(f, scale)
        dg = torch.randn_like(g)
        g.backward(dg)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert not any(n.startswith("Cijk") for n in names), names
    fr = f.detach().clone().requires_grad_()
    gr = gram_ref(fr, scale)
    gr.backward(dg)
    assert _err(g, gr) < 5e-5
    assert _err(f.grad, fr.grad) < 5e-5
