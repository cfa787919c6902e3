"""ConvReLUSequential (VGG features): Conv2d -> ReLU pairs fused into the conv epilogue must be
indistinguishable from the plain Sequential -- outputs, slices, and what hooks observe."""
import pytest
import torch
import torch.nn.functional as F

from torchbooster_amd.models.vgg import vgg16
from torchbooster_amd.ops.conv import ConvReLUSequential


def _plain(f, x, upto):
    for m in list(f)[:upto]:
        x = m(x) if not isinstance(m, torch.nn.Conv2d) else F.conv2d(x, m.weight, m.bias, padding=1)
        if isinstance(m, torch.nn.ReLU):
            x = F.relu(x)
    return x


def test_vgg_features_fused_pairs_match_plain_sequential_cpu():
    torch.manual_seed(0)
    f = vgg16().features
    assert isinstance(f, ConvReLUSequential) and isinstance(f[:7], ConvReLUSequential)
    x = torch.randn(2, 3, 32, 32)
    for upto in (1, 2, 3, 5, 7, 10):
        assert torch.allclose(f[:upto](x), _plain(f, x, upto), atol=1e-5), upto


def test_hooked_modules_see_unfused_values_cpu():
    """offline.yml hooks conv outputs (pre-ReLU), online.yml hooks ReLU outputs."""
    torch.manual_seed(0)
    f = vgg16().features
    got = {}
    f[0].register_forward_hook(lambda m, i, o: got.__setitem__("conv0", o.detach().clone()))
    f[3].register_forward_hook(lambda m, i, o: got.__setitem__("relu3", o.detach().clone()))
    x = torch.randn(1, 3, 16, 16)
    f[:5](x)
    assert torch.allclose(got["conv0"], F.conv2d(x, f[0].weight, f[0].bias, padding=1), atol=1e-5)
    assert got["conv0"].min() < 0  # really pre-activation
    assert torch.allclose(got["relu3"], _plain(f, x, 4), atol=1e-5)


@pytest.mark.gpu
def test_vgg_fused_conv_relu_native_forward_backward():
    """Native bf16 VGG-16 block (fused conv+ReLU epilogue, masked backward) against the same
    module run as a plain Sequential (unfused native convs + ATen ReLU)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.manual_seed(0)
    f = vgg16().features[:9].cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    plain = torch.nn.Sequential(*list(f))
    x = torch.randn(4, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_()
    x2 = x.clone().requires_grad_()
    y1, y2 = f(x1), plain(x2)
    assert ((y1.float() - y2.float()).abs().max() / y2.float().abs().max()).item() < 1e-2
    g = torch.randn_like(y1)
    w = f[2].weight
    gw1, = torch.autograd.grad(y1, [w], g, retain_graph=True)
    gw2, = torch.autograd.grad(y2, [w], g, retain_graph=True)
    assert ((gw1.float() - gw2.float()).abs().max() / gw2.float().abs().max()).item() < 2e-2
    y1.backward(g)
    y2.backward(g)
    assert ((x1.grad.float() - x2.grad.float()).abs().max() / x2.grad.float().abs().max()).item() < 2e-2
