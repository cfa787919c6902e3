"""Weight gradient of the RGB-side 4x4 / stride-2 / pad-1 convs (csrc/conv_tinyin_wgrad.hip): the
DCGAN discriminator's input conv (3 -> 64) and the generator's output transposed conv (64 -> 3)
against fp32 PyTorch on the same bf16 values, and through the autograd paths that route to it.
Reference: examples/img_gen/gan/gan.py (DCGAN D / G edge layers)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("N,P", [(128, 64), (3, 64), (1, 5)])
def test_tinyin_wgrad_matches_fp32(N, P):
    torch.manual_seed(0)
    T = _cl(torch.randn(N, 3, 2 * P, 128, device="cuda").to(torch.bfloat16))
    G = _cl(torch.randn(N, 64, P, 64, device="cuda").to(torch.bfloat16))
    dw = native().conv2d_wgrad_tinyin(T, G)
    ref = torch.nn.grad.conv2d_weight(T.float(), (64, 3, 4, 4), G.float(), stride=2, padding=1)
    assert dw.shape == (64, 3, 4, 4) and dw.is_contiguous(memory_format=torch.channels_last)
    err = ((dw.float() - ref).norm() / ref.norm()).item()
    assert err < 5e-3, err


def test_tinyin_routes_dcgan_edge_layers():
    """The D input conv and the G output transposed conv (native modules) produce weight
    gradients that match fp32 autograd; the tuner is offered the tinyin kernel for both."""
    from torchbooster_amd.ops import conv as CV

    torch.manual_seed(1)
    conv = CV.Conv2d(3, 64, 4, 2, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    convt = CV.ConvTranspose2d(64, 3, 4, 2, 1, bias=False).cuda().to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    x = _cl(torch.randn(16, 3, 128, 128, device="cuda").to(torch.bfloat16))
    z = _cl(torch.randn(16, 64, 64, 64, device="cuda").to(torch.bfloat16))
    for mod, inp in ((conv, x), (convt, z)):
        out = mod(inp)
        g = _cl(torch.randn_like(out))
        out.backward(g)
        ref_mod = (torch.nn.Conv2d(3, 64, 4, 2, 1, bias=False) if mod is conv
                   else torch.nn.ConvTranspose2d(64, 3, 4, 2, 1, bias=False)).cuda()
        ref_mod.weight.data.copy_(mod.weight.detach().float())
        ref_mod(inp.float()).backward(g.float())
        err = ((mod.weight.grad.float() - ref_mod.weight.grad).norm() / ref_mod.weight.grad.norm()).item()
        assert err < 1e-2, (type(mod).__name__, err)
    keys = [k for k in CV.autotune_table() if k[0] == "wgrad" and (64, 3, 4, 4) in k]
    assert keys, CV.autotune_table().keys()


def test_window_gemm_head_is_native():
    """The DCGAN discriminator head (1024x4x4 -> 1, window = whole input) runs as ONE native GEMM
    with the bias in its epilogue (no library GEMM), matching fp32."""
    from torchbooster_amd.ops import conv as CV

    torch.manual_seed(2)
    x = _cl(torch.randn(128, 1024, 4, 4, device="cuda").to(torch.bfloat16))
    w = _cl((torch.randn(1, 1024, 4, 4, device="cuda") * 0.02).to(torch.bfloat16))
    b = torch.randn(1, device="cuda").to(torch.bfloat16)
    y = CV._window_gemm(x, w, b)
    ref = F.conv2d(x.float(), w.float(), b.float())
    assert y.shape == (128, 1, 1, 1)
    assert ((y.float() - ref).norm() / ref.norm()).item() < 1e-2
