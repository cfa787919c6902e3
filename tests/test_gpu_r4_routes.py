"""Native kernels for the shapes the shipped route table used to send to MIOpen:
the bf16 few-pixel forward (VGG-19 512@32² at batch 1, the perceptual loss of the style-transfer
examples, ref examples/img_stt/online/online.py -> torchvision vgg19 features) on the split-
reduction kernel (csrc/conv.hip conv_fwd_splitk_bf16).  Numerics against fp32 PyTorch."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402


@pytest.mark.parametrize("N,C,K,H,bias,relu", [(1, 512, 512, 32, True, False), (1, 512, 512, 16, True, True),
                                               (1, 256, 512, 32, False, False), (2, 512, 256, 14, True, True),
                                               (1, 64, 128, 9, True, False)])
def test_conv_fwd_splitk_bf16(N, C, K, H, bias, relu):
    torch.manual_seed(0)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, 3, 3, device="cuda") / (3 * C ** 0.5)).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    b = torch.randn(K, device="cuda") if bias else None
    assert native().conv_fwd_splitk_ksplit(N, C, K, 3, 3, H, H) > 1
    y = native().conv2d_fwd_splitk(x, w, b, 1, 1, relu)
    ref = F.conv2d(x.float(), w.float(), b, 1, 1)
    if relu:
        ref = F.relu(ref)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    # fixed-order split sum: bitwise repeatable
    assert torch.equal(y, native().conv2d_fwd_splitk(x, w, b, 1, 1, relu))


@pytest.mark.parametrize("N,C,K,H,up,reflect", [(8, 64, 32, 128, 2, True), (2, 64, 32, 40, 2, True),
                                                (3, 128, 96, 24, 1, False), (2, 64, 32, 20, 4, True)])
def test_conv_wgrad_virtual_k32(N, C, K, H, up, reflect):
    """The 32-row dY tile of the virtual-input weight gradient (csrc/conv_wgrad.hip, 64-B LDS rows):
    dW of conv(pad(upsample(x, up), 1, reflect|zero), w) vs fp32 autograd of the same graph."""
    torch.manual_seed(0)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xv = F.interpolate(x.float(), scale_factor=up, mode="nearest") if up > 1 else x.float()
    xv = F.pad(xv, (1, 1, 1, 1), mode="reflect" if reflect else "constant")
    P = xv.shape[2] - 2
    dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.zeros(K, C, 3, 3, device="cuda", requires_grad=True)
    F.conv2d(xv, w).backward(dy.float())
    dw = native().conv2d_wgrad_virtual(dy, x, 3, 3, 1, 1, up, reflect)
    ref = w.grad
    err = (dw.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
