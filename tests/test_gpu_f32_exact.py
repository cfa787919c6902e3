"""IEEE-fp32 convolutions on request.  The fp32 style-transfer examples run at
the reference precision (/root/reference/examples/img_stt/offline/offline.py:103-118, no autocast);
by default their convs use split-bf16 MFMA (~16 mantissa bits, finer than the TF32 cuDNN may use for
fp32 convs).  ``torch.backends.cudnn.allow_tf32 = False`` -- PyTorch's switch that forbids reduced
precision for fp32 convolutions -- makes the native path use the exact-f32 MFMA
(v_mfma_f32_16x16x4_f32): forward, input and weight gradients within 1e-6 (normwise) of a float64
reference, where the split-bf16 default is measurably coarser."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import conv as CV  # noqa: E402


def _rel(a, b):
    return ((a.double().cpu() - b.double()).norm() / b.double().norm()).item()


def _run(x, w, stride, pad, up, reflect, dy=None):
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    y = CV.conv2d_any(xr, wr, None, stride, pad, up, reflect)
    if dy is None:
        dy = torch.randn_like(y)
    y.backward(dy)
    return y.detach(), xr.grad, wr.grad, dy


def _ref(x, w, stride, pad, up, reflect, dy):
    xd = x.detach().cpu().double().requires_grad_()
    wd = w.detach().cpu().double().requires_grad_()
    v = F.interpolate(xd, scale_factor=up, mode="nearest") if up > 1 else xd
    if pad:
        v = F.pad(v, (pad,) * 4, mode="reflect" if reflect else "constant")
    y = F.conv2d(v, wd, stride=stride)
    y.backward(dy.cpu().double())
    return y.detach(), xd.grad, wd.grad


@pytest.mark.parametrize("N,C,H,K,R,stride,pad,up,reflect", [
    (2, 64, 24, 128, 3, 1, 1, 1, False),   # VGG-style 3x3
    (2, 32, 20, 64, 3, 2, 1, 1, False),    # StyleNet downsampling conv
    (2, 64, 12, 32, 3, 1, 1, 2, True),     # DeconvIN: upsample x2 + reflect pad
    (2, 3, 32, 32, 9, 1, 4, 1, True),      # StyleNet RGB input conv 9x9
])
def test_allow_tf32_false_gives_ieee_fp32(N, C, H, K, R, stride, pad, up, reflect):
    torch.manual_seed(N + C + H + K + R)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).contiguous(memory_format=torch.channels_last)
    old = torch.backends.cudnn.allow_tf32
    try:
        torch.backends.cudnn.allow_tf32 = False
        assert CV.f32_exact()
        y, dx, dw, dy = _run(x, w, stride, pad, up, reflect)
        ry, rdx, rdw = _ref(x, w, stride, pad, up, reflect, dy)
        errs = (_rel(y, ry), _rel(dx, rdx), _rel(dw, rdw))
        assert max(errs) < 1e-6, errs
        torch.backends.cudnn.allow_tf32 = True
        if not CV._F32_EXACT_ENV:
            assert not CV.f32_exact()
            ys, dxs, dws, _ = _run(x, w, stride, pad, up, reflect, dy)
            # the default (split-bf16, ~16 mantissa bits) is close, but coarser than the exact path
            split_errs = (_rel(ys, ry), _rel(dxs, rdx), _rel(dws, rdw))
            assert max(split_errs) < 1e-4, split_errs
            print("exact", errs, "split-bf16", split_errs)
    finally:
        torch.backends.cudnn.allow_tf32 = old
