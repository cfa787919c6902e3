"""Standalone native activations (ops/act.py, csrc/aux_ops.hip act_fwd_k / act_bwd_k) against
fp32 ATen, NCHW and channels_last, and the DCGAN discriminator's LeakyReLU running on them."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops.act import activation  # noqa: E402


@pytest.mark.parametrize("act,slope", [("leaky_relu", 0.2), ("relu", 0.0), ("gelu", 0.0), ("silu", 0.0)])
@pytest.mark.parametrize("cl", [False, True])
def test_activation_matches_fp32(act, slope, cl):
    torch.manual_seed(0)
    x = torch.randn(4, 16, 10, 12, device="cuda") * 3
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    xb = x.to(torch.bfloat16).requires_grad_(True)
    y = activation(xb, act, slope)
    g = torch.randn_like(x)
    y.backward(g.to(torch.bfloat16))
    xf = xb.detach().float().requires_grad_(True)
    ref = {"leaky_relu": lambda t: F.leaky_relu(t, slope), "relu": F.relu, "gelu": F.gelu, "silu": F.silu}[act](xf)
    ref.backward(g.to(torch.bfloat16).float())
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item() + 1e-3
    assert (xb.grad.float() - xf.grad).abs().max().item() <= 1e-2 * xf.grad.abs().max().item() + 1e-3


def test_dcgan_discriminator_has_no_aten_activation_kernel():
    from torch.profiler import ProfilerActivity, profile

    from torchbooster_amd.models.dcgan import DCGANDiscriminator

    d = DCGANDiscriminator().cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 128, 128, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    d(x).float().sum().backward()  # warm-up (routing)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        d(x).float().sum().backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert any("act_fwd_k" in n for n in names), names
    assert not any("leaky_relu" in n for n in names), [n for n in names if "leaky" in n]
