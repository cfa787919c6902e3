"""1x1 stride-1 conv weight gradients on the GEMM route (ops/conv.py ``_wgrad`` "gemm" candidate:
dW[K][C] = dyᵀ x over the N*H*W pixel rows on csrc/gemm8.hip's TN kernel or another tuned tile),
written through the zero-copy gradient slot like the conv kernel's, against fp32 ATen."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import conv as CV  # noqa: E402
from torchbooster_amd.ops import gemm as G  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("N,C,H,K", [(8, 256, 14, 1024), (16, 1024, 14, 256), (8, 512, 7, 2048), (4, 64, 28, 256)])
def test_wgrad_gemm_route_matches_fp32(N, C, H, K):
    torch.manual_seed(C + K)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    conv = CV.Conv2d(C, K, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    old = CV._FORCE["wgrad"]
    CV._FORCE["wgrad"] = "gemm"
    G._TILE[("tn", K, C, N * H * H)] = (16, 2)  # pin the TN 8-phase kernel, split 2
    try:
        y = conv(x)
        g = torch.randn_like(y)
        y.backward(g)
    finally:
        CV._FORCE["wgrad"] = old
        G._TILE.pop(("tn", K, C, N * H * H), None)
    ref = torch.ops.aten.convolution_backward(g.float(), x.float(), conv.weight.float(), None, [1, 1], [0, 0],
                                              [1, 1], False, [0, 0], 1, [False, True, False])[1]
    assert conv.weight.grad.shape == ref.shape
    assert _rel(conv.weight.grad, ref) < 8e-3
