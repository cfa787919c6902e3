"""The 8-phase 256x256 NT GEMM (csrc/gemm8.hip, tile 16) against an fp32 PyTorch
reference: full tiles, ragged P / Q tails, odd k-tile counts (the zero-page tail
stagings), every epilogue, and a check that the kernel actually ran."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402

C = native()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _kernels(fn):
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return [e.name for e in prof.events() if e.device_type.name == "CUDA"]


@pytest.mark.parametrize("P,Q,K", [(512, 512, 64), (512, 256, 128), (1000, 520, 192), (300, 72, 320),
                                   (2048, 768, 768), (257, 264, 3072)])
def test_gemm8_matches_fp32(P, Q, K):
    torch.manual_seed(P + Q + K)
    x = (torch.rand(P, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(Q, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    names = _kernels(lambda: C.gemm(x, w, False, tile=16))
    assert any("gemm8_k" in n for n in names), names
    y = C.gemm(x, w, False, tile=16)[0]
    ref = x.float() @ w.float().t()
    assert y.shape == (P, Q)
    assert _rel(y, ref) < 6e-3


@pytest.mark.parametrize("epi", [1, 2, 3, 4, 6, 7])
def test_gemm8_epilogues(epi):
    torch.manual_seed(epi)
    P, Q, K = 700, 384, 256
    x = (torch.rand(P, K, device="cuda") - 0.5).to(torch.bfloat16)
    w = (torch.rand(Q, K, device="cuda") - 0.5).to(torch.bfloat16)
    b = (torch.rand(Q, device="cuda") - 0.5).to(torch.bfloat16)
    r = (torch.rand(P, Q, device="cuda") - 0.5).to(torch.bfloat16)
    z = x.float() @ w.float().t()
    kw = {}
    if epi in (1, 2, 3):
        kw["bias"] = b
        z = z + b.float()
    if epi in (3, 4):
        kw["residual"] = r
        z = z + r.float()
    if epi == 6:
        kw["bias"] = b
        z = z + b.float()
    outs = C.gemm(x, w, False, epi=epi, want_z=epi == 2, tile=16, **kw)
    if epi in (6, 7):
        z = torch.relu(z)
    if epi == 2:
        assert _rel(outs[1], z) < 6e-3
        z = torch.nn.functional.gelu(z)
    assert _rel(outs[0], z) < 6e-3


@pytest.mark.parametrize("P,Q,M,splits", [(256, 256, 64, 1), (768, 3072, 2048, 8), (3072, 768, 1024, 4),
                                          (520, 264, 640, 3), (2304, 768, 3200, 5), (64, 1000 // 8 * 8, 192, 2)])
def test_gemm8_tn_weight_gradient_matches_fp32(P, Q, M, splits):
    """TN variant (transposing LDS reads, split-K partials): dW = dyᵀ x over M rows."""
    torch.manual_seed(P + Q + M)
    dy = (torch.rand(M, P, device="cuda") * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(M, Q, device="cuda") * 2 - 1).to(torch.bfloat16)
    names = _kernels(lambda: C.gemm(dy, x, True, tx=True, tile=16, splits=splits))
    assert any("gemm8_k" in n for n in names), names
    y = C.gemm(dy, x, True, tx=True, tile=16, splits=splits)[0]
    ref = dy.float().t() @ x.float()
    assert y.shape == (P, Q)
    assert _rel(y, ref) < 6e-3


def test_gemm8_tn_ragged_reduction_falls_back_correctly():
    """M % 64 != 0: tile 16 hands the TN product to the split-half tile 10 (same numerics)."""
    torch.manual_seed(7)
    dy = (torch.rand(3152, 512, device="cuda") * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(3152, 264, device="cuda") * 2 - 1).to(torch.bfloat16)
    y = C.gemm(dy, x, True, tx=True, tile=16, splits=4)[0]
    assert _rel(y, dy.float().t() @ x.float()) < 6e-3


@pytest.mark.parametrize("P,K,Q", [(700, 256, 384), (25216 // 8, 768, 3072), (1000, 3072, 768)])
def test_gemm8_nn_input_gradient_matches_fp32(P, K, Q):
    """NN mode (W [K][Q] read transposed from LDS, LDS-staged epilogue): dx = dy w."""
    torch.manual_seed(P + K)
    dy = (torch.rand(P, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(K, Q, device="cuda") * 2 - 1).to(torch.bfloat16)
    names = _kernels(lambda: C.gemm(dy, w, True, tile=16))
    assert any("gemm8_k" in n for n in names), names
    y = C.gemm(dy, w, True, tile=16)[0]
    assert _rel(y, dy.float() @ w.float()) < 6e-3


@pytest.mark.parametrize("tile", [17, 18])
@pytest.mark.parametrize("mode,epi", [("nt", 0), ("nt", 1), ("nt", 2), ("nt", 3), ("nn", 0)])
def test_gemm8_whole_rounds_plus_tail(tile, mode, epi):
    """Tiles 17 / 18 (csrc/gemm.hip): the 8-phase kernel over the rows that fill whole rounds of the
    256 CUs + the 128x128 tile over the rest -- a 25216 x 768 product is 297 256^2 tiles (ViT-B/16
    b128's N = 768 GEMMs).  Every epilogue against fp32, with the tail rows checked on their own."""
    torch.manual_seed(tile * 10 + epi)
    P, Q, K = 25216, 768, 256
    x = (torch.rand(P, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(Q, device="cuda") - 0.5).to(torch.bfloat16)
    r = (torch.rand(P, Q, device="cuda") - 0.5).to(torch.bfloat16)
    if mode == "nt":
        w = (torch.rand(Q, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        kw = dict(bias=b if epi in (1, 2, 3) else None, residual=r if epi == 3 else None, epi=epi,
                  want_z=epi == 2)
        outs = C.gemm(x, w, False, tile=tile, splits=1, **kw)
        z = x.float() @ w.float().t()
        names = _kernels(lambda: C.gemm(x, w, False, tile=tile, splits=1, **kw))
    else:
        w = (torch.rand(K, Q, device="cuda") * 2 - 1).to(torch.bfloat16)
        outs = C.gemm(x, w, True, tile=tile, splits=1)
        z = x.float() @ w.float()
        names = _kernels(lambda: C.gemm(x, w, True, tile=tile, splits=1))
    assert any("gemm8_k" in n for n in names) and any("gemm_k" in n for n in names), names
    if epi in (1, 2, 3):
        z = z + b.float()
    if epi == 3:
        z = z + r.float()
    ref = torch.nn.functional.gelu(z) if epi == 2 else z
    y = outs[0]
    assert _rel(y, ref) < 8e-3
    assert _rel(y[-3000:], ref[-3000:]) < 8e-3
    if epi == 2:
        assert _rel(outs[1], z) < 8e-3
