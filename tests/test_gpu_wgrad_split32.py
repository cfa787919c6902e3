"""fp32 conv weight gradients as split-bf16 passes of the MFMA weight-gradient kernel
(csrc/conv_wgrad.hip conv_wgrad_split32): plain, strided and over the virtual reflect-padded /
upsampled input, against fp32 ATen (error far below the TF32 cuDNN applies by default)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402


def _virtual(x, pad, up, reflect):
    if up > 1:
        x = F.interpolate(x, scale_factor=up, mode="nearest")
    return F.pad(x, (pad,) * 4, mode="reflect" if reflect else "constant")


@pytest.mark.parametrize("N,C,H,K,R,stride,pad,up,reflect", [
    (2, 64, 32, 128, 3, 1, 1, 1, False), (2, 128, 32, 64, 3, 2, 1, 1, False), (2, 64, 16, 64, 3, 1, 1, 2, True),
    (4, 128, 20, 128, 3, 1, 1, 1, True), (2, 64, 24, 128, 1, 1, 0, 1, False)])
def test_wgrad_split32_matches_fp32(N, C, H, K, R, stride, pad, up, reflect):
    torch.manual_seed(C + K + R)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, R, device="cuda") * 0.05
    xv = _virtual(x, pad, up, reflect)
    y = F.conv2d(xv, w, None, stride)
    dy = torch.randn_like(y).contiguous(memory_format=torch.channels_last)
    got = native().conv2d_wgrad_split32(dy, x, R, R, stride, pad, up, reflect)
    with torch.backends.cudnn.flags(allow_tf32=False):
        ref = torch.ops.aten.convolution_backward(dy.double(), xv.double(), w.double(), None, [stride] * 2, [0, 0],
                                                  [1, 1], False, [0, 0], 1, [False, True, False])[1]
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.shape == ref.shape and err < 5e-5, err


@pytest.mark.parametrize("N,C,H,K,R,stride,pad,bias,relu", [
    (2, 64, 32, 128, 3, 1, 1, True, True), (2, 128, 20, 64, 3, 2, 1, False, False), (1, 256, 16, 512, 3, 1, 1, True, False),
    (2, 64, 24, 64, 1, 1, 0, False, True),
    # few output pixels: the reduction split over workgroups (conv_fwd_split32_ksplit), incl. uneven splits
    (1, 512, 16, 512, 3, 1, 1, True, True), (1, 512, 32, 512, 3, 1, 1, False, False), (1, 128, 12, 256, 3, 1, 1, True, True)])
def test_fwd_split32_matches_fp64(N, C, H, K, R, stride, pad, bias, relu):
    torch.manual_seed(C + K + R)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).contiguous(memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda") if bias else None
    C_ = native()
    xh, xl = C_.split_bf16(x)
    wh, wl = C_.split_bf16(w)
    got = C_.conv2d_fwd_split32(xh, xl, wh, wl, b, stride, pad, relu)
    ref = F.conv2d(x.double(), w.double(), None if b is None else b.double(), stride, pad)
    if relu:
        ref = ref.relu()
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.shape == ref.shape and err < 5e-5, err


def test_vgg_fp32_conv_routes_split32_and_grads_match():
    """A frozen fp32 VGG-style block through the native Conv2d: split32 forward / input gradient
    (forced) against fp64 autograd."""
    from torchbooster_amd.ops import conv as CV

    torch.manual_seed(3)
    conv = CV.Conv2d(128, 128, 3, padding=1).cuda().to(memory_format=torch.channels_last)
    conv.requires_grad_(False)
    x = torch.randn(2, 128, 24, 24, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    old = dict(CV._FORCE)
    CV._FORCE["fwd"], CV._FORCE["dgrad"] = "split32", "split32"
    try:
        y = conv(x)
        g = torch.randn_like(y)
        y.backward(g)
    finally:
        CV._FORCE.update(old)
    xd = x.detach().double().requires_grad_(True)
    yd = F.conv2d(xd, conv.weight.double(), conv.bias.double(), 1, 1)
    yd.backward(g.double())
    assert ((y.double() - yd).norm() / yd.norm()).item() < 5e-5
    assert ((x.grad.double() - xd.grad).norm() / xd.grad.norm()).item() < 5e-5


@pytest.mark.parametrize("N,C,H,K,R,pad,up,reflect", [(2, 32, 40, 3, 9, 4, 1, True), (2, 64, 20, 3, 3, 1, 2, True),
                                                      (1, 32, 32, 16, 9, 4, 1, False)])
def test_narrow_wgrad_split32_matches_fp64(N, C, H, K, R, pad, up, reflect):
    """fp32 RGB-head weight gradients as split-bf16 runs of the halo-tile kernel."""
    torch.manual_seed(K + R)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, R, device="cuda") * 0.05
    xv = _virtual(x, pad, up, reflect)
    dy = torch.randn_like(F.conv2d(xv, w)).contiguous(memory_format=torch.channels_last)
    got = native().conv_narrow_wgrad_split32(dy, x, R, R, pad, up, reflect)
    ref = torch.ops.aten.convolution_backward(dy.double(), xv.double(), w.double(), None, [1, 1], [0, 0], [1, 1],
                                              False, [0, 0], 1, [False, True, False])[1]
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.shape == ref.shape and err < 5e-5, err


@pytest.mark.parametrize("N,C,H,K,R,stride,pad,reflect,relu", [(2, 3, 40, 32, 9, 1, 4, True, False),
                                                                (2, 3, 33, 64, 3, 1, 1, False, True),
                                                                (2, 3, 32, 16, 4, 2, 1, False, False)])
def test_tiny32_fwd_matches_fp64(N, C, H, K, R, stride, pad, reflect, relu):
    """fp32 RGB input convs (StyleNet 9x9 3->32, VGG 3->64) as the split-bf16 im2col-gather kernel."""
    torch.manual_seed(K + R)
    x = torch.rand(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.1).contiguous(memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda")
    got = native().conv_tiny32_fwd(x, w, b, stride, pad, reflect, relu)
    xd = F.pad(x.double(), (pad,) * 4, mode="reflect") if reflect else F.pad(x.double(), (pad,) * 4)
    ref = F.conv2d(xd, w.double(), b.double(), stride)
    if relu:
        ref = ref.relu()
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.dtype == torch.float32 and got.shape == ref.shape and err < 5e-5, err


@pytest.mark.parametrize("N,C,H,K,R,pad,up,reflect", [(2, 32, 40, 3, 9, 4, 1, True), (2, 64, 20, 3, 3, 1, 2, True),
                                                      (2, 64, 33, 3, 3, 1, 1, False)])
def test_narrow32_fwd_matches_fp64(N, C, H, K, R, pad, up, reflect):
    """fp32 RGB heads / 3-channel input gradients as three split-bf16 halo-tile runs."""
    torch.manual_seed(C + R)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).contiguous(memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda")
    got = native().conv_narrow_fwd_split32(x, w, b, pad, up, reflect)
    xd = x.double()
    if up > 1:
        xd = F.interpolate(xd, scale_factor=up, mode="nearest")
    xd = F.pad(xd, (pad,) * 4, mode="reflect") if reflect else F.pad(xd, (pad,) * 4)
    ref = F.conv2d(xd, w.double(), b.double())
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.dtype == torch.float32 and got.shape == ref.shape and err < 5e-5, err


def test_fp32_rgb_input_conv_routes_native_and_grads_match():
    """A trainable fp32 VGG-style input conv (3 -> 64) through the native Conv2d with the tiny32
    forward and the narrow32 input gradient forced, against fp64 autograd."""
    from torchbooster_amd.ops import conv as CV

    torch.manual_seed(5)
    conv = CV.Conv2d(3, 64, 3, padding=1).cuda().to(memory_format=torch.channels_last)
    x = torch.rand(2, 3, 36, 36, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    old = dict(CV._FORCE)
    CV._FORCE["fwd"], CV._FORCE["dgrad"] = "tiny32", "narrow32"
    try:
        y = conv(x)
        g = torch.randn_like(y)
        y.backward(g)
    finally:
        CV._FORCE.update(old)
    xd = x.detach().double().requires_grad_(True)
    yd = F.conv2d(xd, conv.weight.double(), conv.bias.double(), 1, 1)
    yd.backward(g.double())
    assert ((y.double() - yd).norm() / yd.norm()).item() < 5e-5
    assert ((x.grad.double() - xd.grad).norm() / xd.grad.norm()).item() < 5e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,C,H,K,R,pad,reflect,relu", [(2, 3, 40, 32, 9, 4, True, False),
                                                        (2, 3, 33, 64, 3, 1, False, True),
                                                        (1, 1, 21, 16, 5, 2, False, False)])
def test_tinyhalo_fwd_matches_fp64(dtype, N, C, H, K, R, pad, reflect, relu):
    """Stride-1 RGB/grey input convs from an LDS halo tile (fp32 split-bf16, or bf16)."""
    torch.manual_seed(K + R + C)
    x = torch.rand(N, C, H, H, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(dtype).contiguous(memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda")
    got = native().conv_tinyhalo_fwd(x, w, b, pad, reflect, relu)
    xd = F.pad(x.double(), (pad,) * 4, mode="reflect") if reflect else F.pad(x.double(), (pad,) * 4)
    ref = F.conv2d(xd, w.double(), b.double())
    if relu:
        ref = ref.relu()
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.dtype == dtype and got.shape == ref.shape and err < (5e-5 if dtype == torch.float32 else 8e-3), err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("N,C,H,K,R,pad,reflect", [(2, 3, 40, 32, 9, 4, True), (2, 3, 33, 64, 3, 1, False),
                                                   (1, 1, 21, 16, 5, 2, False)])
def test_tinyhalo_wgrad_matches_fp64(dtype, N, C, H, K, R, pad, reflect):
    """Weight gradient of the stride-1 RGB/grey input conv from an LDS halo tile."""
    torch.manual_seed(K + R + C + 1)
    x = torch.rand(N, C, H, H, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    P = H + 2 * pad - R + 1
    dy = torch.randn(N, K, P, P, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    got = native().conv_tinyhalo_wgrad(dy, x, R, R, pad, reflect)
    xd = F.pad(x.double(), (pad,) * 4, mode="reflect") if reflect else F.pad(x.double(), (pad,) * 4)
    ref = torch.nn.grad.conv2d_weight(xd, (K, C, R, R), dy.double())
    err = ((got.double() - ref).norm() / ref.norm()).item()
    assert got.dtype == dtype and got.shape == ref.shape and err < (5e-5 if dtype == torch.float32 else 8e-3), err
