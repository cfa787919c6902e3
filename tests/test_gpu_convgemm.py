"""Native im2col / col2im + native GEMM convolutions (ops/convgemm.py, csrc/im2col.hip) against
plain PyTorch fp32 references, at (scaled-down) versions of the shapes that used to route to
MIOpen: StyleNet's 9x9 3->32 reflect-padded input conv, the upsample + reflect-pad 64->32 conv,
DCGAN's 4x4/2 discriminator input and generator output (transposed), VGG-19 at batch 1."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import convgemm as CG  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _virtual(x, pad, up, reflect):
    if up > 1:
        x = F.interpolate(x, scale_factor=up, mode="nearest")
    if pad:
        x = F.pad(x, (pad,) * 4, mode="reflect" if reflect else "constant")
    return x


def _cl(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _kernels(fn):
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return [e.name for e in prof.events() if e.device_type.name == "CUDA"]


@pytest.mark.parametrize("N,C,H,K,R,st,pad,up,reflect,bias,relu", [
    (2, 3, 40, 32, 9, 1, 4, 1, True, True, False),     # StyleNet input conv (reflect 4)
    (2, 64, 16, 32, 3, 1, 1, 2, True, False, False),   # DeconvIN: upsample x2 + reflect 1
    (2, 3, 32, 64, 4, 2, 1, 1, False, False, False),   # DCGAN D input 4x4/2
    (1, 512, 8, 512, 3, 1, 1, 1, False, True, True),   # VGG-19 b1 512-ch (+ fused ReLU)
])
def test_conv_fwd_wgrad_dgrad(N, C, H, K, R, st, pad, up, reflect, bias, relu):
    torch.manual_seed(N * C + H + K)
    x = torch.randn(N, C, H, H, device="cuda")
    w = torch.randn(K, C, R, R, device="cuda") * (1.0 / (C * R * R) ** 0.5)
    b = torch.randn(K, device="cuda") if bias else None
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    ypre = F.conv2d(_virtual(xr, pad, up, reflect), wr, b, st)
    yr = F.relu(ypre) if relu else ypre
    y = CG.conv_fwd(_cl(x), _cl(w), None if b is None else b.to(torch.bfloat16), st, pad, up, reflect, relu)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, yr) < 1.5e-2
    dy = torch.randn_like(yr)
    yr.backward(dy)
    if relu:  # the gradient that reaches the conv is masked by the fused ReLU
        dy = dy * (ypre > 0)
    dw = CG.conv_wgrad(_cl(dy), _cl(x), w.shape, st, pad, up, reflect)
    assert dw.shape == w.shape and _rel(dw, wr.grad) < 2e-2
    if up == 1 and not reflect:
        dx = CG.conv_dgrad(_cl(dy), _cl(w), x.shape, st, pad)
        assert dx.shape == x.shape and _rel(dx, xr.grad) < 2e-2


def test_conv_transpose_fwd_wgrad():
    """DCGAN generator output: ConvTranspose2d(64 -> 3, 4, 2, 1)."""
    torch.manual_seed(9)
    x = torch.randn(2, 64, 16, 16, device="cuda")
    w = torch.randn(64, 3, 4, 4, device="cuda") * 0.05
    b = torch.randn(3, device="cuda")
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = F.conv_transpose2d(xr, wr, b, 2, 1)
    y = CG.convT_fwd(_cl(x), _cl(w), b.to(torch.bfloat16), 2, 1)
    assert y.shape == yr.shape and _rel(y, yr) < 1.5e-2
    dy = torch.randn_like(yr)
    yr.backward(dy)
    dw = CG.convT_wgrad(_cl(x), _cl(dy), w.shape, 2, 1)
    assert dw.shape == w.shape and _rel(dw, wr.grad) < 2e-2
    names = _kernels(lambda: CG.convT_fwd(_cl(x), _cl(w), b.to(torch.bfloat16), 2, 1))
    assert any("col2im_k" in n for n in names) and any("gemm" in n for n in names), names
    assert not any("igemm" in n or "naive_conv" in n or n.startswith("Cijk") for n in names), names
