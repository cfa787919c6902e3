"""Native dense GEMM engine (csrc/gemm.hip) vs an fp32 PyTorch reference.

Covers both weight orientations (x Wᵀ for Linear forward / 1x1 conv, x W for
the input gradient read through transposed LDS loads), every tile
configuration, the fused epilogues (bias, bias+GELU with the saved
pre-activation, bias+residual, residual) and ragged P / Q / K tails."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("tile", list(range(10)))
@pytest.mark.parametrize("tw", [False, True])
@pytest.mark.parametrize("P,Q,K", [(1000, 384, 320), (256, 512, 768), (97, 136, 72)])
def test_gemm_tiles_orientations(tile, tw, P, Q, K):
    torch.manual_seed(P + Q + K + tile)
    x = torch.randn(P, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(Q, K, device="cuda").to(torch.bfloat16) / K ** 0.5
    ref = x.float() @ w.float().t()
    wa = w.t().contiguous() if tw else w
    y = native().gemm(x, wa, tw, tile=tile)[0]
    assert y.shape == (P, Q)
    assert _rel(y, ref) < 1e-2, _rel(y, ref)


@pytest.mark.parametrize("epi", [1, 2, 3, 4])
@pytest.mark.parametrize("tw", [False, True])
def test_gemm_epilogues(epi, tw):
    torch.manual_seed(epi)
    P, Q, K = 777, 512, 256
    x = torch.randn(P, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Q, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(Q, device="cuda").to(torch.bfloat16)
    r = torch.randn(P, Q, device="cuda").to(torch.bfloat16)
    z = x.float() @ w.float().t()
    if epi in (1, 2, 3):
        z = z + b.float()
    if epi in (3, 4):
        z = z + r.float()
    want = F.gelu(z) if epi == 2 else z
    out = native().gemm(x, w.t().contiguous() if tw else w, tw, bias=b if epi in (1, 2, 3) else None,
                        residual=r if epi in (3, 4) else None, epi=epi, want_z=True)
    assert _rel(out[0], want) < 1e-2
    if epi == 2:
        assert _rel(out[1], z) < 1e-2


def test_gemm_strided_rows_and_out():
    torch.manual_seed(5)
    big = torch.randn(300, 1024, device="cuda").to(torch.bfloat16)
    x = big[:, 128:128 + 512]  # row stride 1024
    w = torch.randn(256, 512, device="cuda").to(torch.bfloat16)
    out = torch.empty(300, 256, device="cuda", dtype=torch.bfloat16)
    native().gemm(x, w, False, out=out)
    assert _rel(out, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("tile", [0, 3, 5, 8])
@pytest.mark.parametrize("splits", [1, 3])
def test_gemm_transposed_x_split_k(tile, splits):
    """dW = dYᵀ X (both operands reduction-major, split-K over the rows)."""
    torch.manual_seed(tile + 10 * splits)
    M, N, Kin = 2000, 320, 192
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, Kin, device="cuda").to(torch.bfloat16)
    ref = dy.float().t() @ x.float()
    got = native().gemm(dy, x, True, tx=True, tile=tile, splits=splits)[0]
    assert got.shape == (N, Kin)
    assert _rel(got, ref) < 1e-2


def test_linear_ops_with_ragged_feature_counts():
    """LeNet's 120 -> 84 -> 10 head and a 1-logit head: padded to multiples of 8."""
    from torchbooster_amd.ops import gemm as G

    torch.manual_seed(9)
    for (M, K, Q) in ((256, 120, 84), (256, 84, 10), (64, 512, 1)):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Q, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(Q, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, Q, device="cuda").to(torch.bfloat16)
        assert _rel(G.mm_nt(x, w, b), x.float() @ w.float().t() + b.float()) < 1e-2
        assert _rel(G.mm_nn(dy, w), dy.float() @ w.float()) < 1e-2
        assert _rel(G.mm_tn(dy, x), dy.float().t() @ x.float()) < 1e-2
