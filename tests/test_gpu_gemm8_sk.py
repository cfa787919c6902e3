"""Tail split-K of the 8-phase 256x256 GEMM (csrc/gemm8.hip sk_splits): a partial last round of
tiles (the N = 768 ViT-B/16 products: 297 tiles on 256 CUs) runs as k-ranges whose f32 partials
the last arrival sums in split order.  Numerics against fp32 PyTorch for the NT (Linear forward,
every epilogue) and NN (input gradient) forms; run-to-run bitwise stable; equal to the unsplit
kernel to float rounding.  Reference layer: nn.Linear."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402

TILE8 = 16


def _r(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


@pytest.mark.parametrize("P,Q,K", [(25216, 768, 768), (25216, 768, 3072), (12800, 1280, 512)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("S", [2, 3])
def test_gemm8_nt_tail_split(P, Q, K, epi, S):
    torch.manual_seed(0)
    x = _r(P, K)
    w = _r(Q, K, scale=K ** -0.5)
    b = _r(Q) if epi in (1, 2, 3) else None
    res = _r(P, Q) if epi == 3 else None
    outs = native().gemm(x, w, False, bias=b, residual=res, epi=epi, want_z=epi == 2, tile=TILE8, splits=S)
    base = native().gemm(x, w, False, bias=b, residual=res, epi=epi, want_z=epi == 2, tile=TILE8, splits=1)
    ref = x.float() @ w.float().t()
    if b is not None:
        ref = ref + b.float()
    if res is not None:
        ref = ref + res.float()
    if epi == 2:
        assert torch.allclose(outs[1].float(), ref, rtol=2e-2, atol=2e-2)
        ref = F.gelu(ref)
    err = (outs[0].float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err
    # same products as the unsplit kernel up to the f32 summation order
    d = (outs[0].float() - base[0].float()).abs().max().item()
    assert d <= 1e-2 * ref.abs().max().item() + 1e-2, d
    again = native().gemm(x, w, False, bias=b, residual=res, epi=epi, want_z=epi == 2, tile=TILE8, splits=S)
    assert torch.equal(again[0], outs[0])


@pytest.mark.parametrize("P,Q,K", [(25216, 768, 2304), (25216, 768, 3072), (25216, 768, 768)])
@pytest.mark.parametrize("S", [2, 3])
def test_gemm8_nn_tail_split(P, Q, K, S):
    torch.manual_seed(1)
    dy = _r(P, K)
    w = _r(K, Q, scale=K ** -0.5)  # [out, in]: y = dy w
    y = native().gemm(dy, w, True, tile=TILE8, splits=S)[0]
    ref = dy.float() @ w.float()
    err = (y.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err
    assert torch.equal(native().gemm(dy, w, True, tile=TILE8, splits=S)[0], y)


def test_vit_linear_layers_native_only(monkeypatch):
    """The ViT-B/16 block's four N = 768 products through ops.gemm with the library candidate
    off: the tuner picks among native tiles (tail split included) and matches fp32."""
    from torchbooster_amd.ops import gemm as G

    monkeypatch.setattr(G, "_BLAS_CANDIDATE", False)
    torch.manual_seed(2)
    x = _r(25216, 3072)
    w = _r(768, 3072, scale=3072 ** -0.5)
    b = _r(768)
    y = G.mm_nt(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    assert (y.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 1e-2
