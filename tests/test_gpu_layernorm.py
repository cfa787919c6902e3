"""LayerNorm row kernels (csrc/layernorm.hip) vs plain PyTorch fp32.

Covers every row-group layout the launcher picks: compile-time (R, NCH) pairs
(C = 192/256/384/512/768/1024/1280/1536/2048/3072/4096), the runtime-R generic
kernel (C = 2304, 64, 8), row counts that leave a partial last group, the fused
residual add (forward) and residual-stream gradient add (backward)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import _ext  # noqa: E402
from torchbooster_amd.ops.norm import layer_norm  # noqa: E402

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    _ext.native()


def _err(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


SHAPES = [(25216, 768), (1001, 768), (3, 768), (999, 384), (517, 192), (333, 256), (77, 512), (129, 1024),
          (41, 1280), (17, 1536), (9, 2048), (11, 3072), (5, 4096), (23, 2304), (70, 64), (13, 8)]


@pytest.mark.parametrize("M,C", SHAPES)
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("res", [False, True])
def test_layer_norm_fwd_bwd(M, C, dt, res):
    torch.manual_seed(M + C)
    x = (torch.randn(M, C, device=DEV) * 2 + 0.5).to(dt).requires_grad_()
    r = torch.randn(M, C, device=DEV).to(dt).requires_grad_() if res else None
    w = (torch.rand(C, device=DEV) + 0.5).requires_grad_()
    b = torch.randn(C, device=DEV).requires_grad_()
    out = layer_norm(x, w, b, 1e-5, r)
    y, xs = out if res else (out, None)

    xf = x.detach().float().requires_grad_()
    rf = r.detach().float().requires_grad_() if res else None
    wf, bf = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    xsf = xf + rf if res else xf
    yf = F.layer_norm(xsf, (C,), wf, bf, 1e-5)

    tol = 1e-2 if dt == torch.bfloat16 else 1e-5
    assert y.dtype == dt and _err(y, yf) < tol
    if res:
        assert _err(xs, xsf) < tol
    dy = torch.randn(M, C, device=DEV)
    loss = (y.float() * dy).sum()
    lossf = (yf * dy).sum()
    if res:  # the residual stream is consumed downstream too: exercises the fused dadd
        ds = torch.randn(M, C, device=DEV)
        loss = loss + (xs.float() * ds).sum()
        lossf = lossf + (xsf * ds).sum()
    loss.backward()
    lossf.backward()
    assert _err(x.grad, xf.grad) < 2 * tol
    if res:
        assert _err(r.grad, rf.grad) < 2 * tol
    assert _err(w.grad, wf.grad) < 2 * tol
    assert _err(b.grad, bf.grad) < 2 * tol


def test_layer_norm_deterministic():
    x = torch.randn(4099, 768, device=DEV, dtype=torch.bfloat16)
    w = torch.rand(768, device=DEV)
    b = torch.randn(768, device=DEV)
    dy = torch.randn(4099, 768, device=DEV, dtype=torch.bfloat16)
    C = _ext.native()
    y, _, mean, rstd = C.ln_forward(x, None, w, b, 1e-5)
    outs = [C.ln_backward(dy, x, w, mean, rstd) for _ in range(3)]
    for o in outs[1:]:
        for a, c in zip(outs[0], o):
            assert torch.equal(a, c)
