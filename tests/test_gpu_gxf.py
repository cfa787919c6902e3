"""Deferred BN backward apply (ops/norm.py BnGradXf, csrc/conv.hip GXF).

The BatchNorm after a 1x1 stride-1 conv no longer writes its input gradient: its backward runs the
finalize only, and the conv's input gradient applies dX = ka * act'(z) * g + c0 + c1 * x to its
operand as it lands in LDS (storing dX once for the weight gradient).

* kernel: ``conv2d_dgrad_gxf`` against a plain fp32 PyTorch reference of the same op (the BN
  backward apply, rounded to bf16 like the kernel's operand, then the 1x1 input gradient, the
  residual addend, the next BN's partial sums, the materialised dX);
* model: ResNet-50 gradients with and without the deferral agree to within bf16 rounding, the
  apply pass is really gone, and a bottleneck matches an fp32 autograd reference.

Reference: the torchvision BatchNorm2d backward of the img_cls example
(/root/reference/examples/img_cls/resnet/resnet.py:44-68,111).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.models import resnet as R  # noqa: E402
from torchbooster_amd.ops import _ext  # noqa: E402
from torchbooster_amd.ops import norm as N  # noqa: E402

DEV = torch.device("cuda", 0)


def _bits(mask_bool):
    """[M, C] bool -> [M, C/8] bytes (bit k of byte j = channel 8 j + k)."""
    M, C = mask_bool.shape
    b = mask_bool.view(M, C // 8, 8).to(torch.int32)
    w = (1 << torch.arange(8, device=mask_bool.device, dtype=torch.int32))
    return (b * w).sum(-1).to(torch.uint8)


def _rows(t):
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("gxf,add,bnb", [(2, 0, 1), (1, 2, 2), (1, 1, 2), (1, 1, 0)])
@pytest.mark.parametrize("C,K,n,hw", [(256, 64, 3, 13), (64, 256, 2, 15), (512, 128, 2, 9), (128, 256, 1, 11)])
def test_dgrad_gxf_kernel_vs_fp32(gxf, add, bnb, C, K, n, hw):
    nat = _ext.native()
    torch.manual_seed(C + K + gxf)
    g = torch.randn(n, C, hw, hw, device=DEV).to(torch.bfloat16)
    xb = torch.randn(n, C, hw, hw, device=DEV).to(torch.bfloat16)
    w = (torch.randn(C, K, 1, 1, device=DEV) * 0.1).to(torch.bfloat16)  # the conv: K -> C channels
    wt = w.permute(1, 0, 2, 3).contiguous()  # the flipped / transposed dgrad weight [K, C, 1, 1]
    coef = torch.randn(3, C, device=DEV) * torch.tensor([[1.0], [0.1], [0.05]], device=DEV)
    scale = torch.randn(C, device=DEV)
    shift = torch.randn(C, device=DEV) * 0.5
    gr, xr = _rows(g).float(), _rows(xb).float()
    if gxf == 1:
        keep = (xr * scale + shift) > 0
        bits = None
    else:
        keep = torch.rand(gr.shape, device=DEV) > 0.4
        bits = _bits(keep)
    dz = coef[0] * torch.where(keep, gr, torch.zeros_like(gr)) + coef[1] + coef[2] * xr
    dz_b = dz.to(torch.bfloat16)  # the kernel's operand is the bf16-rounded transform
    M = gr.shape[0]
    dx_ref = dz_b.float() @ w.view(C, K).float()  # [M, K]
    addend = amask = None
    if add:
        addend = torch.randn(n, K, hw, hw, device=DEV).to(torch.bfloat16)
        ar = _rows(addend).float()
        if add == 2:
            akeep = torch.rand(M, K, device=DEV) > 0.5
            amask = _bits(akeep)
            ar = torch.where(akeep, ar, torch.zeros_like(ar))
        dx_ref = dx_ref + ar
    bx = bsc = bsf = bmu = bbits = None
    if bnb:
        bx = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        bmu = torch.randn(K, device=DEV) * 0.1
        if bnb == 2:
            bkeep = torch.rand(M, K, device=DEV) > 0.5
            bbits = _bits(bkeep)
        else:
            bsc, bsf = torch.randn(K, device=DEV), torch.randn(K, device=DEV) * 0.5
    dx, part, dzo = nat.conv2d_dgrad_gxf(_cl(g), wt, None if addend is None else _cl(addend), amask, bnb, bx, bsc,
                                         bsf, bmu, bbits, gxf, _cl(xb), bits, scale if gxf == 1 else None,
                                         shift if gxf == 1 else None, coef.contiguous(), True)
    torch.cuda.synchronize()
    dxr = _rows(dx).float()
    err = ((dxr - dx_ref).norm() / dx_ref.norm()).item()
    assert err < 1e-2, err
    # the materialised BN input gradient is the bf16 transform itself (up to fma contraction)
    dzr = _rows(dzo).float()
    assert ((dzr - dz_b.float()).abs() <= 1e-2 * dz_b.float().abs() + 1e-3).all()
    if bnb:
        # partial sums of the next BN over the bf16 dX: (sum dz', sum dz' (xb - mean))
        dv = dxr  # (the kernel's own bf16 output)
        if bnb == 2:
            dzz = torch.where(bkeep, dv, torch.zeros_like(dv))
        else:
            dzz = torch.where(bx.float() * bsc + bsf > 0, dv, torch.zeros_like(dv))
        want = torch.stack([dzz.sum(0), (dzz * (bx.float() - bmu)).sum(0)])
        got = part.sum(0)
        assert torch.allclose(got, want, rtol=2e-3, atol=1e-3 * want.abs().max().item()), (got - want).abs().max()


def _grads(model, x, on, monkeypatch):
    monkeypatch.setattr(N, "_GXF", on)
    model.zero_grad(set_to_none=True)
    out = model(x).float()
    out.square().mean().backward()
    torch.cuda.synchronize()
    g = {n: p.grad.detach().float().clone() for n, p in model.named_parameters() if p.grad is not None}
    g["__out__"] = out.detach()
    return g


def test_resnet50_gradients_match_without_deferral(monkeypatch):
    """Deferral on vs off: same logits, gradients equal to within the partial-sum grouping (the GXF
    dgrad's 64-pixel tiles sum the next BN's partials in a different order)."""
    _ext.native()
    torch.manual_seed(0)
    model = R.resnet50(num_classes=16).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = _cl(torch.randn(4, 3, 64, 64, device=DEV, dtype=torch.bfloat16))
    off = _grads(model, x, False, monkeypatch)
    on = _grads(model, x, True, monkeypatch)
    assert on.keys() == off.keys()
    assert torch.equal(on["__out__"], off["__out__"])
    d = {n: ((on[n] - off[n]).norm() / off[n].norm().clamp_min(1e-12)).item() for n in on}
    print("relative gradient differences (deepest first):")
    for n in reversed(list(d)):
        print(f"  {n:40s} {d[n]:.2e}")
    # the classifier and the last stage see (almost) the same gradients: the grouping of the partial
    # sums is the only difference there
    for n in d:
        if n.startswith(("fc.", "layer4.2.", "layer4.1.")):
            assert d[n] < 1e-3, (n, d[n])
    assert max(d.values()) < 2e-1, max(d.items(), key=lambda t: t[1])


def test_apply_pass_is_deferred(monkeypatch):
    """With the deferral, bn1 of every bottleneck and bn3 of every identity block run no apply: their
    conv's backward receives the placeholder and consumes the link."""
    _ext.native()
    monkeypatch.setattr(N, "_GXF", True)
    torch.manual_seed(0)
    model = R.resnet50(num_classes=16).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = _cl(torch.randn(2, 3, 64, 64, device=DEV, dtype=torch.bfloat16))
    calls = {"coef": 0, "gxf": 0, "materialize": 0}
    nat = _ext.native()
    real_coef, real_gxf = nat.bn_backward_coef, nat.conv2d_dgrad_gxf
    real_mat = N.BnGradXf.materialize

    class Spy:
        def __getattr__(self, k):
            if k == "bn_backward_coef":
                def f(*a, **kw):
                    calls["coef"] += 1
                    return real_coef(*a, **kw)
                return f
            if k == "conv2d_dgrad_gxf":
                def f(*a, **kw):
                    calls["gxf"] += 1
                    return real_gxf(*a, **kw)
                return f
            return getattr(nat, k)

    def mat(self):
        calls["materialize"] += 1
        return real_mat(self)

    spy = Spy()
    from torchbooster_amd.ops import conv as CV
    monkeypatch.setattr(N, "native", lambda: spy)
    monkeypatch.setattr(CV, "native", lambda: spy)
    monkeypatch.setattr(N.BnGradXf, "materialize", mat)
    model(x).float().square().mean().backward()
    torch.cuda.synchronize()
    # 16 bottlenecks: bn1 everywhere (16) + bn3 of the 12 identity blocks, except the last block
    # whose output BN feeds the pool (no partials): 16 + 11
    # (== 27 on the shipped routes; a route without the BN partial epilogue leaves its BN undeferred)
    assert calls["coef"] >= 24, calls
    assert calls["gxf"] == calls["coef"] and calls["materialize"] == 0, calls


def _ref_bottleneck(blk, x, wf):
    """fp32 autograd reference (training-mode BN); ``wf``: fp32 leaf copies of the parameters."""
    def cba(m, t, act=True):
        c = m.conv
        z = F.conv2d(t, wf[id(c.weight)], None, c.stride, c.padding)
        z = F.batch_norm(z, None, None, wf[id(m.bn.weight)], wf[id(m.bn.bias)], True, 0.0, m.bn.eps)
        return z.relu() if act else z

    h = cba(blk.c1, x)
    h = cba(blk.c2, h)
    h = cba(blk.c3, h, act=False)
    idn = x if blk.down is None else cba(blk.down, x, act=False)
    return (h + idn).relu()


class _Pair(torch.nn.Module):
    """Two identity bottlenecks: the second one's conv1 dgrad supplies the first one's bn3 partials,
    so both deferrals (bn1 and bn3 of the first block) run."""

    def __init__(self, ch):
        super().__init__()
        self.b1 = R.Bottleneck(4 * ch, ch, 1)
        self.b2 = R.Bottleneck(4 * ch, ch, 1)

    def forward(self, x):
        h, link = self.b1.forward_linked(x)
        return self.b2.forward_linked(h, link)[0]


@pytest.mark.parametrize("ch,hw", [(64, 14), (128, 9)])
def test_bottleneck_pair_vs_fp32(monkeypatch, ch, hw):
    """Input and weight gradients of two chained bottlenecks against fp32 autograd: the deferral is
    no worse than the written-apply path."""
    _ext.native()
    torch.manual_seed(ch)
    m = _Pair(ch).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    x0 = torch.randn(4, 4 * ch, hw, hw, device=DEV).to(torch.bfloat16)
    params = dict(m.named_parameters())
    wf = {id(p): p.detach().float().requires_grad_(True) for p in params.values()}
    xr = x0.float().requires_grad_(True)
    ref = _ref_bottleneck(m.b2, _ref_bottleneck(m.b1, xr, wf), wf)
    gy = torch.randn_like(ref)
    leaves = [xr] + [wf[id(p)] for p in params.values()]
    gref = torch.autograd.grad(ref, leaves, gy)
    errs = {}
    for on in (False, True):
        monkeypatch.setattr(N, "_GXF", on)
        m.zero_grad(set_to_none=True)
        x = _cl(x0).requires_grad_(True)
        out = m(x).float()
        (out * gy).sum().backward()
        torch.cuda.synchronize()
        got = [x.grad] + [p.grad for p in params.values()]
        errs[on] = [((a.float() - b).norm() / b.norm().clamp_min(1e-12)).item() for a, b in zip(got, gref)]
    for i, (e_on, e_off) in enumerate(zip(errs[True], errs[False])):
        assert e_on < max(1.5 * e_off, 2e-2), (i, e_on, e_off)
