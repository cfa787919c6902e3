"""Linear / Linear+GELU native backward pieces (csrc/colsum.hip) vs plain PyTorch fp32."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import _ext  # noqa: E402
from torchbooster_amd.ops.linear import Linear, LinearGELU  # noqa: E402

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    _ext.native()


def _err(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,C,dt", [(25216, 768, torch.bfloat16), (37, 64, torch.float32), (1000, 3072, torch.bfloat16),
                                    (5, 8, torch.bfloat16)])
def test_colsum(M, C, dt):
    x = torch.randn(M, C, device=DEV).to(dt)
    got = _ext.native().colsum(x)
    assert got.dtype == dt
    assert _err(got, x.float().sum(0)) < (1e-2 if dt == torch.bfloat16 else 1e-5)


def test_gelu_bwd_colsum():
    torch.manual_seed(1)
    z = torch.randn(333, 256, device=DEV).to(torch.bfloat16)
    dy = torch.randn(333, 256, device=DEV).to(torch.bfloat16)
    dz, db = _ext.native().gelu_bwd_colsum(dy, z)
    zr = z.float().requires_grad_()
    F.gelu(zr).backward(dy.float())
    assert _err(dz, zr.grad) < 1e-2
    assert _err(db, zr.grad.sum(0)) < 1e-2


def _kernels(fn):
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return [e.name for e in prof.events() if e.device_type.name == "CUDA"]


@pytest.fixture
def native_gemm_only(monkeypatch):
    """The autotuner may keep hipBLASLt for a shape; pin the native engine for this test."""
    from torchbooster_amd.ops import gemm as G

    monkeypatch.setattr(G, "_BLAS_CANDIDATE", False)
    monkeypatch.setattr(G, "_TILE", {})
    yield


@pytest.mark.parametrize("cls", [Linear, LinearGELU])
def test_linear_modules_match_fp32(cls, native_gemm_only):
    torch.manual_seed(2)
    m = cls(192, 384).to(DEV).to(torch.bfloat16)
    ref = torch.nn.Linear(192, 384).to(DEV)
    ref.load_state_dict({k: v.float() for k, v in m.state_dict().items()})
    x = torch.randn(4, 50, 192, device=DEV).to(torch.bfloat16).requires_grad_()
    xr = x.detach().float().requires_grad_()
    y = m(x)
    yr = ref(xr)
    if cls is LinearGELU:
        yr = F.gelu(yr)
    g = torch.randn_like(yr)
    names = _kernels(lambda: y.backward(g.to(y.dtype)))
    names += _kernels(lambda: m(x))
    yr.backward(g)
    assert any("gemm_k" in n or "gemm8_k" in n for n in names), names  # the native engine ran
    assert not any(n.startswith("Cijk") for n in names), names  # ... and not hipBLASLt
    assert _err(y, yr) < 1e-2
    assert _err(x.grad, xr.grad) < 2e-2
    assert _err(m.weight.grad, ref.weight.grad) < 2e-2
    assert _err(m.bias.grad, ref.bias.grad) < 2e-2


def test_linear_gelu_double_backward():
    """create_graph (GAN gradient penalty) goes through a differentiable path."""
    m = LinearGELU(16, 16).to(DEV)
    x = torch.randn(8, 16, device=DEV, requires_grad=True)
    (g,) = torch.autograd.grad(m(x).sum(), x, create_graph=True)
    g.pow(2).sum().backward()
    assert m.weight.grad is not None and torch.isfinite(m.weight.grad).all()


@pytest.mark.parametrize("tile", [116, 117, 118])
def test_linear_dgrad_on_cached_transposed_weight(tile, monkeypatch):
    """mm_nn's NT candidates (tiles TRANS + 16 .. 18): dX = dY W on the cached Wᵀ (ops/conv.py
    transposed_linear_weight) against fp32, and the cached copy follows the fused optimizer's
    in-place update (refreshed with the flip cache after the step)."""
    from torchbooster_amd.ops import gemm as G
    from torchbooster_amd.ops.linear import Linear
    from torchbooster_amd.ops.optim import FusedAdamW

    torch.manual_seed(tile)
    lin = Linear(768, 384).cuda().to(torch.bfloat16)
    opt = FusedAdamW(lin.parameters(), lr=1e-2)
    x = (torch.rand(25216, 768, device="cuda") - 0.5).to(torch.bfloat16).requires_grad_()
    monkeypatch.setitem(G._TILE, ("nn", 25216, 768, 384), (tile, 1))
    for step in range(2):
        opt.zero_grad(set_to_none=True)
        x.grad = None
        y = lin(x)
        g = (torch.rand_like(y) - 0.5)
        y.backward(g)
        ref = g.float() @ lin.weight.detach().float()
        assert ((x.grad.float() - ref).norm() / ref.norm()).item() < 8e-3, step
        opt.step()  # rewrites the weight in place: the next step must see the new W through the cache
