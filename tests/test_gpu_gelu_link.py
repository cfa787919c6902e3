"""ViT MLP backward with the fc2 -> fc1 GELU hand-off (ops/linear.py GeluLink, csrc/gemm8.hip NN
mode + GELU-backward epilogue): every gradient matches the unfused native path and fp32 ATen."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.models.vit import MLP  # noqa: E402
from torchbooster_amd.ops import linear as L  # noqa: E402
from torchbooster_amd.ops._ext import native  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("transposed", [False, True])
def test_gemm_nn_gelu_bwd_matches_fp32(transposed):
    """NN kernel (transposing LDS reads of w) and the NT kernel on wᵀ (the cached transposed weight of
    ops/linear.py) against fp32."""
    torch.manual_seed(0)
    P, K, Q = 1000, 256, 1024
    dy = (torch.rand(P, K, device="cuda") - 0.5).to(torch.bfloat16)
    w = (torch.rand(K, Q, device="cuda") - 0.5).to(torch.bfloat16)
    z = (torch.rand(P, Q, device="cuda") * 4 - 2).to(torch.bfloat16)
    dz, db = native().gemm_nn_gelu_bwd(dy, w, z, None, w.t().contiguous() if transposed else None)
    zf = z.float()
    gp = 0.5 * (1 + torch.erf(zf * 0.7071067811865476)) + zf * torch.exp(-0.5 * zf * zf) * 0.3989422804014327
    ref = (dy.float() @ w.float()) * gp
    assert _rel(dz, ref) < 6e-3
    assert _rel(db, dz.float().sum(0)) < 1e-2


@pytest.mark.parametrize("fuse", [True, False])
def test_mlp_gradients_with_and_without_link(fuse):
    torch.manual_seed(1)
    m = MLP(256, 1024).cuda().to(torch.bfloat16)
    ref = MLP(256, 1024).cuda()
    ref.load_state_dict({k: v.float() for k, v in m.state_dict().items()})
    x = torch.randn(4, 197, 256, device="cuda")
    xb = x.to(torch.bfloat16).requires_grad_(True)
    xf = x.clone().requires_grad_(True)
    old = L._FUSE_GELU_BWD
    L._FUSE_GELU_BWD = fuse
    try:
        y = m(xb)
        g = torch.randn_like(y)
        y.backward(g)
    finally:
        L._FUSE_GELU_BWD = old
    yf = ref(xf)
    yf.backward(g.float())
    assert _rel(xb.grad, xf.grad) < 2e-2
    for (n, p), (_, pf) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, pf.grad) < 2e-2, n
