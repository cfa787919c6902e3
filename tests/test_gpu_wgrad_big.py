"""Big-tile conv weight gradient (csrc/conv_wgrad.hip conv_wgrad_big_k: 8 waves, 256 x 256 /
256 x 128 / 128 x 256 output tiles, a 2-3 stage direct-to-LDS ring, split-K partials + the
deterministic reduce, or the bf16 output directly when one split covers the pixels) against the fp32
PyTorch weight gradient, and against the 128 x 128 kernel.  Reference: the conv weight gradients of
examples/img_cls/resnet/resnet.py:111 (cuDNN wgrad there)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402


@pytest.fixture
def big():
    C = native()
    old = C.conv_wgrad_get_big()
    yield C
    C.conv_wgrad_set_big(old)


def _cl(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


# (N, C, H, K, R, stride, pad, expected tile)
SHAPES = [
    (32, 256, 14, 256, 1, 1, 0, (256, 256)),    # 1x1, square tile
    (24, 128, 14, 256, 3, 1, 1, (256, 128)),    # 3x3: 1152 weight columns
    (24, 128, 28, 256, 3, 2, 1, (256, 128)),    # 3x3 stride 2 with padded taps
    (24, 256, 14, 128, 1, 1, 0, (128, 256)),    # 128-channel output
    (5, 256, 31, 256, 1, 1, 0, (256, 256)),     # 4,805 pixels: ragged last k-tile
    (8, 256, 23, 256, 3, 1, 1, (256, 256)),     # 3x3 over 256 channels, odd map
    (84, 512, 7, 2048, 3, 1, 1, (256, 256)),    # 2048 x 4608 weight: one split, bf16 stored directly
]


@pytest.mark.parametrize("N,C,H,K,R,st,pad,tile", SHAPES)
def test_wgrad_big_matches_fp32(big, N, C, H, K, R, st, pad, tile):
    torch.manual_seed(N + C + K + R)
    P = (H + 2 * pad - R) // st + 1
    x = _cl(torch.randn(N, C, H, H, device="cuda"))
    dy = _cl(torch.randn(N, K, P, P, device="cuda"))
    big.conv_wgrad_set_big(1)
    assert big.conv_wgrad_big_choice(C, K, R, R, N * P * P) == (tile[0] << 12) | tile[1]
    dw = big.conv2d_wgrad(dy, x, R, R, st, pad)
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, R, R), dy.float(), stride=st, padding=pad)
    err = (dw.float() - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item(), (err, ref.abs().max().item())
    # the 128 x 128 kernel: same products, other summation order
    big.conv_wgrad_set_big(0)
    assert big.conv_wgrad_big_choice(C, K, R, R, N * P * P) == 0
    dw0 = big.conv2d_wgrad(dy, x, R, R, st, pad)
    err0 = (dw0.float() - ref).abs().max().item()
    assert err <= 1.5 * err0 + 1e-3 * ref.abs().max().item(), (err, err0)


def test_wgrad_big_ineligible_shapes_keep_the_small_kernel(big):
    big.conv_wgrad_set_big(1)
    assert big.conv_wgrad_big_choice(64, 64, 3, 3, 802816) == 0      # 64 x 576: no 256 side
    assert big.conv_wgrad_big_choice(128, 128, 3, 3, 200704) == 0    # 128 x 1152: 128 x 128 tiles only
    assert big.conv_wgrad_big_choice(256, 256, 1, 1, 2048) == 0      # too few pixels
    big.conv_wgrad_set_big(0)
    assert big.conv_wgrad_big_choice(256, 256, 1, 1, 1 << 20) == 0


def test_wgrad_big_kernel_runs(big):
    big.conv_wgrad_set_big(1)
    x = _cl(torch.randn(32, 256, 14, 14, device="cuda"))
    dy = _cl(torch.randn(32, 256, 14, 14, device="cuda"))
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        big.conv2d_wgrad(dy, x, 1, 1, 1, 0)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events()]
    assert any("conv_wgrad_big_k" in n for n in names), sorted(set(names))[:20]
