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


@pytest.mark.parametrize("epi", [1, 2, 3, 4])
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
    outs = C.gemm(x, w, False, epi=epi, want_z=epi == 2, tile=16, **kw)
    if epi == 2:
        assert _rel(outs[1], z) < 6e-3
        z = torch.nn.functional.gelu(z)
    assert _rel(outs[0], z) < 6e-3
