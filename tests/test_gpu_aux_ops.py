"""Small fused losses / resampling kernels (csrc/aux_ops.hip) vs plain PyTorch fp32 references.

K16 reflection pad, K17 nearest upsample, K19 total variation, K20 mean/std,
K21 BCE-with-logits + Gaussian KL, K22 hinge.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import _ext  # noqa: E402
from torchbooster_amd.ops import losses as L  # noqa: E402
from torchbooster_amd.ops.resample import reflection_pad2d, upsample_nearest2d  # noqa: E402

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    _ext.native()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _pair(shape, dtype, cl, seed):
    torch.manual_seed(seed)
    x = torch.randn(*shape, device=DEV).to(dtype)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_()
    return x.requires_grad_(), xr


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("shape", [(1, 3, 512, 512), (8, 3, 64, 48), (2, 5, 7, 9)])
def test_total_variation(shape, dtype, cl):
    x, xr = _pair(shape, dtype, cl, sum(shape))
    y = L.total_variation(x)
    yr = L.total_variation_ref(xr)
    assert y.dtype == torch.float32 and y.dim() == 0
    assert abs(y.item() - yr.item()) / abs(yr.item()) < 1e-4
    (2.5 * y).backward()
    (2.5 * yr).backward()
    # sign gradient: integer-valued, exact unless a difference rounds to 0 in bf16
    mism = (x.grad.float() - xr.grad).abs().gt(1e-3).float().mean().item()
    assert mism < (1e-6 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("margin,sign", [(1.0, -1.0), (1.0, 1.0), (0.5, -1.0)])
@pytest.mark.parametrize("n", [256, 4097])
def test_hinge(n, margin, sign, dtype):
    x, xr = _pair((n, 1), dtype, False, n)
    y = L.hinge(x, margin, sign)
    yr = L.hinge_ref(xr, margin, sign)
    assert abs(y.item() - yr.item()) < 1e-5 * max(1.0, abs(yr.item()))
    y.backward()
    yr.backward()
    assert torch.allclose(x.grad.float(), xr.grad, atol=1e-6, rtol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(256, 784), (3, 5)])
def test_bce_with_logits(shape, dtype):
    x, xr = _pair(shape, dtype, False, 3)
    t = torch.rand(*shape, device=DEV).to(dtype)
    y = L.bce_with_logits(x, t)
    yr = F.binary_cross_entropy_with_logits(xr, t.float())
    assert abs(y.item() - yr.item()) < 1e-4 * abs(yr.item())
    (3.0 * y).backward()
    (3.0 * yr).backward()
    assert _rel(x.grad, xr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gaussian_kld(dtype):
    torch.manual_seed(5)
    mu = torch.randn(256, 128, device=DEV).to(dtype).requires_grad_()
    lv = (0.5 * torch.randn(256, 128, device=DEV)).to(dtype).requires_grad_()
    mur, lvr = mu.detach().float().requires_grad_(), lv.detach().float().requires_grad_()
    y = L.gaussian_kld(mu, lv)
    yr = L.gaussian_kld_ref(mur, lvr)
    assert abs(y.item() - yr.item()) < 1e-4 * abs(yr.item())
    y.backward()
    yr.backward()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(mu.grad, mur.grad) < tol and _rel(lv.grad, lvr.grad) < tol


def test_kld_on_chunked_encoder_output():
    torch.manual_seed(6)
    h = torch.randn(64, 256, device=DEV, requires_grad=True)
    mu, lv = h.chunk(2, dim=1)  # non-contiguous views, as in the VAE encoder
    L.gaussian_kld(mu, lv).backward()
    hr = h.detach().clone().requires_grad_()
    mur, lvr = hr.chunk(2, dim=1)
    L.gaussian_kld_ref(mur, lvr).backward()
    assert _rel(h.grad, hr.grad) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cl", [False, True])
@pytest.mark.parametrize("shape", [(32, 64, 32, 32), (2, 512, 8, 8), (3, 70, 5, 7), (1, 3, 1, 2)])
def test_mean_std(shape, dtype, cl):
    x, xr = _pair(shape, dtype, cl, 11)
    with torch.no_grad():
        x += 3.0  # offset mean: exercises the two-pass variance
    xr = x.detach().float().requires_grad_()  # same (rounded) values as the kernel sees
    m, s = L.mean_std(x)
    mr, sr = L.mean_std_ref(xr)
    assert m.shape == mr.shape and s.shape == sr.shape
    tol = 1e-5 if dtype == torch.float32 else 1e-3
    assert _rel(m, mr) < tol and _rel(s, sr) < tol
    gm, gs = torch.randn_like(mr), torch.randn_like(sr)
    ((m * gm).sum() + (s * gs).sum()).backward()
    ((mr * gm).sum() + (sr * gs).sum()).backward()
    assert _rel(x.grad, xr.grad) < (1e-4 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,pads", [((8, 3, 256, 256), (4, 4, 4, 4)), ((2, 128, 64, 64), (1, 1, 1, 1)),
                                        ((1, 5, 6, 7), (2, 3, 1, 4)), ((2, 8, 3, 3), (2, 2, 2, 2))])
def test_reflection_pad(shape, pads, dtype):
    x, xr = _pair(shape, dtype, True, 7)
    y = reflection_pad2d(x, pads)
    yr = F.pad(xr, pads, mode="reflect")
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(y.float(), yr.to(dtype).float())
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    assert _rel(x.grad, xr.grad) < (1e-6 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,f", [((8, 128, 64, 64), 2), ((32, 256, 32, 32), 2), ((2, 3, 5, 7), 3)])
def test_upsample_nearest(shape, f, dtype):
    x, xr = _pair(shape, dtype, True, 9)
    y = upsample_nearest2d(x, f)
    yr = F.interpolate(xr, scale_factor=f, mode="nearest")
    assert y.shape == yr.shape
    assert torch.equal(y.float(), yr.to(dtype).float())
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    assert _rel(x.grad, xr.grad) < (1e-6 if dtype == torch.float32 else 1e-2)


@pytest.mark.gpu
def test_style_stats_loss_native_matches_expanded_reference():
    """The native-statistics AdaIN style loss against the reference formula on the expanded
    fp32 tensors (adain.py:55-58, 134), bf16 channels_last features, values and gradients."""
    from torchbooster_amd.models.style import style_stats_loss

    torch.manual_seed(0)
    shapes = [(4, 64, 32, 32), (4, 128, 16, 16), (4, 512, 4, 4)]
    m = [torch.randn(sh, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
         .requires_grad_() for sh in shapes]
    s = [torch.randn(sh, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
         for sh in shapes]
    mr = [t.detach().float().requires_grad_() for t in m]

    def mu_std_ref(f):
        mu = f.mean(dim=[2, 3], keepdim=True)
        std = f.var(dim=[2, 3], keepdim=True).add(1e-5).sqrt()
        return mu.expand_as(f), std.expand_as(f)

    ref = sum(F.mse_loss(xm, sm) + F.mse_loss(xs, ss)
              for (xm, xs), (sm, ss) in zip(map(mu_std_ref, mr), map(mu_std_ref, [t.float() for t in s])))
    new = style_stats_loss(m, s)
    assert abs(float(new) - float(ref)) <= 1e-4 * abs(float(ref))
    ref.backward()
    new.backward()
    for a, b in zip(m, mr):
        assert _rel(a.grad, b.grad) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_native_gelu_forward(dtype):
    """Native exact-erf GELU pass (ViT fc1 when the GEMM runs on hipBLASLt) vs fp32 F.gelu."""
    torch.manual_seed(0)
    z = (torch.randn(1000, 72, device="cuda") * 3).to(dtype)
    y = _ext.native().gelu_fwd(z)
    ref = F.gelu(z.float())
    assert y.dtype == dtype and y.shape == z.shape
    assert _rel(y, ref) < (1e-5 if dtype == torch.float32 else 1e-2)
