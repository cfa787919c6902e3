"""Generic convolution family (csrc/conv_any.hip) vs an fp32 ATen reference of the same op:
odd channel counts, 5x5 / 9x9 taps, stride 2, reflect padding and nearest upsampling
folded into the addressing; forward, input gradient, weight gradient; fp32 and bf16."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402

# (N, C, H, W, K, R, stride, pad, up, reflect)
CASES = [
    (8, 1, 28, 28, 6, 5, 1, 0, 1, False),      # LeNet conv1
    (8, 6, 12, 12, 16, 5, 1, 0, 1, False),     # LeNet conv2
    (2, 3, 64, 64, 32, 9, 1, 4, 1, True),      # StyleNet in: ReflectionPad(4) + 9x9
    (2, 32, 64, 64, 64, 3, 2, 1, 1, True),     # StyleNet down: reflect pad 1, 3x3 / 2
    (2, 64, 16, 16, 32, 3, 1, 1, 2, True),     # DeconvIN: Upsample(2) + ReflectionPad(1) + 3x3
    (2, 32, 64, 64, 3, 9, 1, 4, 1, True),      # StyleNet out: 32 -> 3, 9x9
    (1, 64, 32, 32, 64, 3, 1, 1, 1, False),    # VGG-style zero pad (fp32 reference precision)
    # strided zero-pad convs: dgrad on stride-phase tiles written straight into dX
    (4, 3, 33, 33, 16, 4, 2, 1, 1, False),     # DCGAN D input (odd size)
    (2, 16, 17, 17, 3, 3, 2, 1, 1, False),     # 3-channel dy: scalar phase gathers
    (2, 8, 16, 16, 24, 5, 2, 2, 1, False),     # 5x5 / 2
    (2, 8, 15, 15, 8, 3, 2, 0, 1, False),      # no padding
    (2, 8, 16, 16, 8, 1, 2, 0, 1, False),      # 1x1 / 2: odd-parity pixels meet no tap
    (2, 3, 16, 16, 8, 3, 3, 1, 1, False),      # stride 3 (9 phases)
]


def _ref(x, w, b, stride, pad, up, reflect):
    if up > 1:
        x = F.interpolate(x, scale_factor=up, mode="nearest")
    if pad:
        x = F.pad(x, (pad,) * 4, mode="reflect" if reflect else "constant")
    return F.conv2d(x, w, b, stride)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.fixture(params=["f32_exact", "f32_split"])
def f32_mode(request):
    """fp32 generic convs on the exact-f32 MFMA and on the split-bf16 MFMA (the default)."""
    C_ = native()
    prev = C_.conv_any_f32_split()
    C_.conv_any_set_f32_split(request.param == "f32_split")
    yield request.param
    C_.conv_any_set_f32_split(prev)


@pytest.mark.parametrize("case", CASES)
def test_conv_any_fp32_modes(case, f32_mode):
    """fp32: exact-f32 MFMA held to 2e-5, split-bf16 (hi + lo, three bf16 MFMAs) to 1e-4 --
    both well inside the TF32 (~5e-4) cuDNN gives the reference's fp32 convs by default."""
    _check_case(case, torch.float32, 2e-5 if f32_mode == "f32_exact" else 1e-4)


@pytest.mark.parametrize("case", CASES)
def test_conv_any_fwd_dgrad_wgrad(case):
    _check_case(case, torch.bfloat16, 1.5e-2)


def _check_case(case, dtype, tol):
    N, C, H, W, K, R, st, pad, up, refl = case
    torch.manual_seed(C * 100 + K)
    x = torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5
    b = torch.randn(K, device="cuda")
    xr, wr, br = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone()
    yr = _ref(xr, wr, br, st, pad, up, refl)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    C_ = native()
    y = C_.conv_any_fwd(x.to(dtype), w.to(dtype), b.to(dtype), st, pad, up, refl)
    assert y.shape == yr.shape and _rel(y, yr) < tol, _rel(y, yr)
    dyd = dy.to(dtype).contiguous(memory_format=torch.channels_last)
    dx = C_.conv_any_dgrad(dyd, w.to(dtype), H, W, st, pad, up, refl)
    assert dx.shape == x.shape and _rel(dx, xr.grad) < tol, _rel(dx, xr.grad)
    dw = C_.conv_any_wgrad(dyd, x.to(dtype), R, R, st, pad, up, refl)
    assert dw.shape == w.shape and _rel(dw, wr.grad) < tol * 2, _rel(dw, wr.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("Ci,Co,R,st,pad,H", [(64, 3, 4, 2, 1, 32), (100, 64, 4, 1, 0, 4), (16, 8, 3, 2, 1, 9)])
def test_conv_transpose_generic(Ci, Co, R, st, pad, H, dtype, f32_mode):
    """DCGAN-style transposed convs with channel counts the 64-channel kernels do not
    take (generator output 64 -> 3, latent 100 -> 64) on the generic family."""
    from torchbooster_amd.ops.conv import ConvTranspose2d

    torch.manual_seed(Ci + Co)
    m = ConvTranspose2d(Ci, Co, R, st, pad).cuda().to(dtype)
    ref = torch.nn.ConvTranspose2d(Ci, Co, R, st, pad).cuda()
    ref.load_state_dict({k: v.float() for k, v in m.state_dict().items()})
    x = torch.randn(4, Ci, H, H, device="cuda")
    xa = x.to(dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    xr = x.clone().requires_grad_()
    y, yr = m(xa), ref(xr)
    tol = (2e-5 if f32_mode == "f32_exact" else 1e-4) if dtype == torch.float32 else 1.5e-2
    assert _rel(y, yr) < tol
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g)
    assert _rel(xa.grad, xr.grad) < tol and _rel(m.weight.grad, ref.weight.grad) < 2 * tol
    assert _rel(m.bias.grad, ref.bias.grad) < 2 * tol


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C", [3, 64, 12])
def test_bias_grad_colsum(C, dtype):
    """conv bias gradients on the native column sum (C % 8 != 0 folded into wider rows)."""
    from torchbooster_amd.ops.conv import _bias_grad

    dy = torch.randn(4, C, 10, 12, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    ref = dy.float().sum(dim=(0, 2, 3))
    got = _bias_grad(dy, dtype)
    assert got.dtype == dtype and _rel(got, ref) < (1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_window_gemm_route(dtype):
    """a conv whose window covers the whole input (DCGAN D head 1024x4x4 -> 1) as one GEMM"""
    from torchbooster_amd.ops.conv import _window_gemm

    torch.manual_seed(0)
    x = torch.randn(16, 256, 4, 4, device="cuda").contiguous(memory_format=torch.channels_last)
    w = (torch.randn(2, 256, 4, 4, device="cuda") / 64).contiguous(memory_format=torch.channels_last)
    b = torch.randn(2, device="cuda")
    ref = F.conv2d(x, w, b)
    got = _window_gemm(x.to(dtype), w.to(dtype), b.to(dtype))
    assert got.shape == ref.shape and _rel(got, ref) < (1e-5 if dtype == torch.float32 else 1e-2)


# (N, C, H, K, R, stride, pad, up, reflect): the 64-channel implicit-GEMM kernels reading the
# virtual input pad(upsample(x)) directly (StyleNet residual blocks, AdaIN decoder DeconvIN)
VIRT = [
    (2, 64, 16, 64, 3, 1, 1, 2, True),
    (2, 128, 17, 128, 3, 1, 1, 1, True),
    (2, 64, 16, 128, 3, 2, 1, 1, True),
    (2, 64, 8, 64, 3, 1, 1, 2, False),
    (1, 64, 9, 64, 5, 1, 2, 4, True),
]


@pytest.mark.parametrize("case", VIRT)
def test_conv64_virtual_input(case):
    N, C, H, K, R, st, pad, up, refl = case
    torch.manual_seed(C + K + H)
    x = torch.randn(N, C, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5
    b = torch.randn(K, device="cuda")
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = _ref(xr, wr, b, st, pad, up, refl)
    dy = torch.randn_like(yr)
    yr.backward(dy)
    C_ = native()
    xb = x.bfloat16().contiguous(memory_format=torch.channels_last)
    wb = w.bfloat16().contiguous(memory_format=torch.channels_last)
    y = C_.conv2d_fwd_virtual(xb, wb, b, st, pad, up, refl)
    assert y.shape == yr.shape and _rel(y, yr) < 1.5e-2, _rel(y, yr)
    dyb = dy.bfloat16().contiguous(memory_format=torch.channels_last)
    dx = C_.conv2d_dgrad_virtual(dyb, C_.conv_flip_weight(wb), H, H, st, pad, up, refl)
    assert dx.shape == x.shape and _rel(dx, xr.grad) < 1.5e-2, _rel(dx, xr.grad)
    dw = C_.conv2d_wgrad_virtual(dyb, xb, R, R, st, pad, up, refl)
    assert dw.shape == w.shape and _rel(dw, wr.grad) < 3e-2, _rel(dw, wr.grad)


# (N, C, H, W, K, R, pad, up, reflect): csrc/conv_narrow.hip (K <= 16, halo tile in LDS)
NARROW = [
    (2, 64, 40, 40, 3, 9, 4, 1, True),     # AdaIN decoder out: ReflectionPad(4) + 9x9, 64 -> 3
    (2, 32, 33, 37, 3, 9, 4, 1, True),     # StyleNet out, ragged tiles: 32 -> 3
    (1, 64, 20, 18, 16, 3, 1, 1, False),   # 16 outputs, zero padding, 3x3
    (2, 32, 9, 11, 5, 5, 2, 2, True),      # upsample x2 folded in, 5x5
    (1, 64, 12, 12, 1, 9, 0, 1, False),    # no padding, output smaller than one tile
]


@pytest.mark.parametrize("case", NARROW)
def test_conv_narrow_forward(case):
    """Narrow-output forward against the fp32 ATen conv on the same bf16 values (route pinned:
    the op is called directly)."""
    N, C, H, W, K, R, pad, up, reflect = case
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda")
    y = native().conv_narrow_fwd(x, w, b.to(torch.bfloat16), pad, up, reflect)
    ref = _ref(x.float(), w.float(), b.to(torch.bfloat16).float(), 1, pad, up, reflect)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err


def test_conv_narrow_is_routed_for_the_style_heads():
    """The autotuner offers the narrow kernel for the decoder RGB head and it wins (the shipped
    route table has no entry for this key, so it is timed here)."""
    from torchbooster_amd.ops import conv as CV

    x = torch.randn(8, 32, 128, 128, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(3, 32, 9, 9, device="cuda") * 0.05).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = CV.conv2d_any(x, w, None, 1, 4, 1, True)
    ref = _ref(x.float(), w.float(), None, 1, 4, 1, True)
    assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    key = ("fwd", "any", tuple(x.shape), tuple(w.shape), str(x.dtype), 1, 4, 1, True, False)
    if CV._AUTOTUNE and not CV._DISABLE:
        assert CV.autotune_table().get(key) == "narrow", CV.autotune_table().get(key)


@pytest.mark.parametrize("case", NARROW)
def test_conv_narrow_weight_gradient(case):
    """Narrow-output weight gradient (halo tiles, transposed-dy MFMA, split-K over pixel tiles)
    against autograd of the fp32 ATen conv on the materialised virtual input."""
    N, C, H, W, K, R, pad, up, reflect = case
    torch.manual_seed(1)
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    P = H * up + 2 * pad - R + 1
    dy = torch.randn(N, K, P, W * up + 2 * pad - R + 1, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dw = native().conv_narrow_wgrad(dy, x, R, R, pad, up, reflect)
    wr = torch.zeros(K, C, R, R, device="cuda", requires_grad=True)
    _ref(x.float(), wr, None, 1, pad, up, reflect).backward(dy.float())
    assert dw.shape == wr.shape
    err = ((dw.float() - wr.grad).abs().max() / wr.grad.abs().max()).item()
    assert err < 1e-2, err


# (N, C, H, W, K, R, stride, pad, reflect): csrc/conv_narrow.hip conv_tinyc_fwd (C*R*S <= 256)
TINYC = [
    (2, 3, 64, 64, 64, 3, 1, 1, False),    # VGG conv1_1
    (2, 3, 33, 35, 64, 4, 2, 1, False),    # DCGAN discriminator input (odd sizes)
    (2, 3, 40, 40, 32, 9, 1, 4, True),     # StyleNet input: ReflectionPad(4) + 9x9 (243 taps)
    (4, 1, 28, 28, 16, 5, 1, 0, False),    # LeNet-style grey input (K padded to 16)
    (1, 6, 12, 12, 16, 5, 1, 0, False),    # 150 taps, K 16
    (2, 3, 16, 16, 128, 3, 1, 1, False),   # two 64-channel workgroup columns
]


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("case", TINYC)
def test_conv_tinyc_forward(case, relu):
    N, C, H, W, K, R, st, pad, reflect = case
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda").to(torch.bfloat16)
    y = native().conv_tinyc_fwd(x, w, b, st, pad, reflect, relu)
    ref = _ref(x.float(), w.float(), b.float(), st, pad, 1, reflect)
    if relu:
        ref = ref.clamp_min(0)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("C,K,R,pad", [(3, 64, 3, 1), (3, 32, 5, 2), (1, 64, 3, 0)])
def test_narrow_input_gradient_route(C, K, R, pad):
    """Input gradient of an RGB-input conv via the halo-tile forward on dy with the flipped,
    transposed weight (route 'narrow' forced) against autograd of the fp32 ATen conv."""
    import os
    from torchbooster_amd.ops import conv as CV

    torch.manual_seed(0)
    x = torch.randn(2, C, 36, 40, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    xr = x.float().requires_grad_()
    yr = F.conv2d(xr, w.float(), None, 1, pad)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    old = CV._FORCE["dgrad"]
    CV._FORCE["dgrad"] = "narrow"
    try:
        xx = x.clone().requires_grad_()
        y = CV.conv2d_any(xx, w, None, 1, pad, 1, False)
        y.backward(dy)
    finally:
        CV._FORCE["dgrad"] = old
    err = ((xx.grad.float() - xr.grad).abs().max() / xr.grad.abs().max()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("Ci,Co,R,st,pad,H", [(64, 3, 4, 2, 1, 32), (32, 3, 4, 2, 1, 17), (64, 16, 3, 2, 1, 9),
                                               (64, 1, 5, 1, 2, 12)])
def test_conv_narrow_transpose_forward(Ci, Co, R, st, pad, H):
    """Stride-phase narrow transposed conv (DCGAN generator RGB head) vs fp32 ATen."""
    torch.manual_seed(0)
    x = torch.randn(2, Ci, H, H + 3, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Ci, Co, R, R, device="cuda") * 0.1).to(torch.bfloat16)
    b = torch.randn(Co, device="cuda").to(torch.bfloat16)
    y = native().conv_narrow_transpose_fwd(x, w, b, st, pad)
    ref = F.conv_transpose2d(x.float(), w.float(), b.float(), st, pad)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-2, err


def test_strided_rgb_input_gradient_via_narrow_transpose():
    """Input gradient of a stride-2 conv with 3 input channels (DCGAN discriminator input) on
    the stride-phase narrow transposed kernel (route forced), vs autograd of fp32 ATen."""
    from torchbooster_amd.ops import conv as CV

    torch.manual_seed(0)
    x = torch.randn(4, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 4, 4, device="cuda") * 0.1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    xr = x.float().requires_grad_()
    yr = F.conv2d(xr, w.float(), None, 2, 1)
    dy = torch.randn_like(yr).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    yr.backward(dy.float())
    old = CV._FORCE["dgrad"]
    CV._FORCE["dgrad"] = "narrow"
    try:
        xx = x.clone().requires_grad_()
        CV.conv2d_any(xx, w, None, 2, 1, 1, False).backward(dy)
    finally:
        CV._FORCE["dgrad"] = old
    err = ((xx.grad.float() - xr.grad).abs().max() / xr.grad.abs().max()).item()
    assert err < 1e-2, err
