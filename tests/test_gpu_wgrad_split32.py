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
