"""Numerics of every native HIP kernel vs a plain PyTorch fp32 reference (MI355X only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops import _ext  # noqa: E402

DEV = "cuda"


@pytest.fixture(autouse=True, scope="module")
def _native_loaded():
    _ext.native()  # fail loudly if the extension did not load


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("shape,act,res,dt", [
    ((8, 64, 14, 14), "relu", True, torch.bfloat16),
    ((4, 6, 12, 12), "gelu", False, torch.float32),
    ((16, 256, 7, 7), "none", False, torch.bfloat16),
    ((2, 48, 9, 9), "silu", True, torch.float32),
    ((3, 40, 5, 5), "leaky_relu", False, torch.float32),
    ((64, 1024), "relu", False, torch.float32),
])
def test_batchnorm_act(shape, act, res, dt):
    from torchbooster_amd.ops.norm import act_ref, batch_norm_act

    torch.manual_seed(0)
    x = (torch.randn(*shape, device=DEV) * 2 + 3).to(dt)
    if x.dim() == 4:
        x = x.contiguous(memory_format=torch.channels_last)
    C = shape[1]
    r = torch.randn_like(x) if res else None
    w = torch.randn(C, device=DEV, requires_grad=True)
    b = torch.randn(C, device=DEV, requires_grad=True)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rm2, rv2 = rm.clone(), rv.clone()
    xa = x.detach().clone().requires_grad_()
    ra = r.detach().clone().requires_grad_() if res else None
    y = batch_norm_act(xa, w, b, rm, rv, True, 0.1, 1e-5, ra, act, 0.2)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if res else None
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    z = F.batch_norm(xr, rm2, rv2, wr, br, True, 0.1, 1e-5)
    if res:
        z = z + rr
    yr = act_ref(z, act, 0.2)
    yr.backward(g.float())
    tol = 2e-2 if dt == torch.bfloat16 else 1e-4
    assert rel(y, yr) < tol
    assert rel(xa.grad, xr.grad) < tol
    assert rel(w.grad, wr.grad) < 1e-3
    assert rel(b.grad, br.grad) < 1e-3
    assert torch.allclose(rm, rm2, atol=1e-4) and torch.allclose(rv, rv2, rtol=1e-3, atol=1e-3)
    if res:
        assert rel(ra.grad, rr.grad) < tol
    # eval mode uses running stats
    ye = batch_norm_act(x, w, b, rm, rv, False, 0.1, 1e-5, None, act, 0.2)
    ze = F.batch_norm(x.float(), rm, rv, w.detach(), b.detach(), False)
    assert rel(ye, act_ref(ze, act, 0.2)) < tol


@pytest.mark.parametrize("N,C,H,G,act,dt", [(2, 64, 9, 64, "gelu", torch.bfloat16), (3, 32, 8, 8, "none", torch.float32),
                                            (8, 128, 16, 32, "silu", torch.bfloat16), (2, 6, 5, 3, "relu", torch.float32)])
def test_groupnorm_act(N, C, H, G, act, dt):
    from torchbooster_amd.ops.norm import act_ref, group_norm_act

    torch.manual_seed(1)
    x = (torch.randn(N, C, H, H, device=DEV) * 3 + 1).to(dt).contiguous(memory_format=torch.channels_last)
    w = torch.randn(C, device=DEV, requires_grad=True)
    b = torch.randn(C, device=DEV, requires_grad=True)
    xa = x.detach().clone().requires_grad_()
    y = group_norm_act(xa, G, w, b, 1e-5, None, act)
    g = torch.randn_like(y)
    y.backward(g)
    xr = x.detach().float().requires_grad_()
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    yr = act_ref(F.group_norm(xr, G, wr, br, 1e-5), act)
    yr.backward(g.float())
    tol = 3e-2 if dt == torch.bfloat16 else 1e-4
    assert rel(y, yr) < tol
    assert rel(xa.grad, xr.grad) < tol
    assert rel(w.grad, wr.grad) < 1e-3 if dt == torch.float32 else rel(w.grad, wr.grad) < 3e-2
    assert rel(b.grad, br.grad) < 1e-3


@pytest.mark.parametrize("K,dt,smooth", [(10, torch.float32, 0.1), (1000, torch.bfloat16, 0.1), (37, torch.float32, 0.0)])
def test_cross_entropy_accuracy(K, dt, smooth):
    from torchbooster_amd.ops.loss import cross_entropy_accuracy

    torch.manual_seed(2)
    lg = torch.randn(300, K, device=DEV).to(dt).requires_grad_()
    lab = torch.randint(0, K, (300,), device=DEV)
    lab[5] = -100
    loss, acc = cross_entropy_accuracy(lg, lab, smooth)
    loss.backward()
    lr_ = lg.detach().float().requires_grad_()
    l2 = F.cross_entropy(lr_, lab, label_smoothing=smooth)
    l2.backward()
    a2 = ((lr_.argmax(-1) == lab).sum() / 300).item()
    assert abs(loss.item() - l2.item()) < 1e-4
    assert abs(acc.item() - a2) < 1e-6
    assert (lg.grad.float() - lr_.grad).abs().max().item() < (1e-6 if dt == torch.float32 else 1e-4)


@pytest.mark.parametrize("pdt", [torch.float32, torch.bfloat16])
def test_fused_adamw_matches_torch(pdt):
    from torchbooster_amd.ops.optim import FusedAdamW

    torch.manual_seed(3)
    shapes = [(1000, 33), (17,), (64, 3, 7, 7)]
    ps = [torch.randn(s, device=DEV) for s in shapes]
    ps[2] = ps[2].contiguous(memory_format=torch.channels_last)
    pa = [p.clone().to(pdt).requires_grad_() for p in ps]
    # f32 reference starting from the same (rounded) values as the low-precision params
    pb = [p.clone().to(pdt).float().requires_grad_() for p in ps]
    oa = FusedAdamW(pa, lr=1e-2, weight_decay=0.1, amsgrad=False)
    ob = torch.optim.AdamW(pb, lr=1e-2, weight_decay=0.1)
    for _ in range(5):
        for a, b in zip(pa, pb):
            g = torch.randn_like(b)
            a.grad = g.to(pdt)
            b.grad = g.to(pdt).float()
        oa.step(clip=1.0)
        torch.nn.utils.clip_grad_norm_(pb, 1.0)
        ob.step()
    for a, b in zip(pa, pb):
        if pdt == torch.float32:
            assert (a - b).abs().max().item() < 1e-5
        else:
            # f32 master weights track torch exactly; the bf16 param is their rounding
            assert (oa.state[a]["master_param"] - b).abs().max().item() < 1e-5
            assert torch.equal(a, oa.state[a]["master_param"].to(torch.bfloat16))
    # state dict round trip keeps f32 moments
    sd = oa.state_dict()
    assert sd["state"][0]["exp_avg"].dtype == torch.float32
    oc = FusedAdamW([p.detach().clone().requires_grad_() for p in pa], lr=1e-2, weight_decay=0.1)
    oc.load_state_dict(sd)
    assert torch.equal(oc.state_dict()["state"][0]["exp_avg"], sd["state"][0]["exp_avg"])


def test_fused_sgd_matches_torch():
    from torchbooster_amd.ops.optim import FusedSGD

    torch.manual_seed(4)
    ps = [torch.randn(s, device=DEV) for s in [(300, 7), (5,)]]
    pa = [p.clone().requires_grad_() for p in ps]
    pb = [p.clone().requires_grad_() for p in ps]
    oa = FusedSGD(pa, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    ob = torch.optim.SGD(pb, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    for _ in range(4):
        for a, b in zip(pa, pb):
            g = torch.randn_like(a)
            a.grad, b.grad = g.clone(), g.clone()
        oa.step()
        ob.step()
    for a, b in zip(pa, pb):
        assert (a - b).abs().max().item() < 1e-5


def test_fused_clip_grad_norm():
    from torchbooster_amd.ops.optim import clip_grad_norm_

    ps = [torch.randn(100, device=DEV, requires_grad=True), torch.randn(7, device=DEV, requires_grad=True)]
    for p in ps:
        p.grad = torch.randn_like(p) * 10
    ref = [p.grad.clone() for p in ps]
    n = clip_grad_norm_(ps, 1.0)
    n2 = torch.norm(torch.stack([r.norm() for r in ref]))
    assert abs(n.item() - n2.item()) / n2.item() < 1e-5
    assert abs(torch.norm(torch.stack([p.grad.norm() for p in ps])).item() - 1.0) < 1e-4


@pytest.mark.parametrize("N,C,H,K,k,s,p", [
    (2, 64, 14, 64, 3, 1, 1), (2, 64, 14, 128, 1, 1, 0), (3, 128, 9, 64, 3, 2, 1), (2, 256, 8, 128, 1, 2, 0),
    (1, 64, 7, 192, 3, 1, 1), (5, 128, 6, 256, 3, 1, 0), (2, 64, 11, 64, 5, 1, 2),
])
def test_native_conv_forward_and_backward(N, C, H, K, k, s, p, monkeypatch):
    """Every direction pinned to the native kernels (no autotuned MIOpen route) and the
    route taken asserted from the kernel names."""
    from torchbooster_amd.ops import conv as nconv
    from torchbooster_amd.ops.conv import conv2d, native_supported

    for d in ("fwd", "dgrad", "wgrad"):
        monkeypatch.setitem(nconv._FORCE, d, "native")
    torch.manual_seed(5)
    x = torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, k, k, device=DEV) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert native_supported(x, w, s, p)
    xa, wa = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = conv2d(xa, wa, None, s, p)
    yr = F.conv2d(x.float(), w.float(), None, s, p)
    assert y.shape == yr.shape
    assert rel(y, yr) < 1e-2
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    F.conv2d(xr, wr, None, s, p).backward(g.float())
    assert rel(xa.grad, xr.grad) < 2e-2
    assert rel(wa.grad, wr.grad) < 2e-2
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        conv2d(xa, wa, None, s, p).backward(g)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type.name == "CUDA"]
    assert any("conv_fwd_k" in n for n in names) and any("conv_wgrad_k" in n for n in names), names
    if s == 1 or k * k <= 16:  # dgrad: native stride-1 / parity-class kernels
        assert not any("igemm" in n or "ck::" in n for n in names), names


@pytest.mark.parametrize("N,C,H,K,k,s,p", [
    (16, 64, 28, 128, 3, 1, 1), (8, 256, 20, 128, 1, 2, 0), (4, 64, 15, 128, 2, 1, 0), (2, 128, 9, 64, 3, 2, 1),
    (32, 64, 56, 64, 1, 1, 0),
])
def test_native_conv_wgrad(N, C, H, K, k, s, p):
    """Weight gradient kernel (split reduction + transposing LDS reads) vs fp32."""
    from torchbooster_amd.ops.conv import conv2d_wgrad

    torch.manual_seed(11)
    x = torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(K, C, k, k, device=DEV)
    P = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, K, P, P, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dw = conv2d_wgrad(dy, x, k, s, p)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), w, None, [s, s], [p, p], [1, 1], False, [0, 0],
                                              1, [False, True, False])[1]
    assert dw.shape == ref.shape and dw.is_contiguous(memory_format=torch.channels_last)
    assert rel(dw, ref) < 1e-2


@pytest.mark.parametrize("in_ch,ch,stride", [(256, 64, 1), (64, 64, 1), (256, 128, 2)])
def test_bottleneck_residual_grad_fusion(in_ch, ch, stride, monkeypatch):
    """Block input gradient = dgrad(c1) + residual grad, summed in the dgrad
    epilogue.  Three BNs in series amplify bf16 rounding, so the native bf16
    block is held to the error of the same block on stock ATen bf16 (both vs
    an fp32 reference)."""
    from torchbooster_amd.models.resnet import Bottleneck

    def relnorm(a, b):
        return ((a.float() - b.float()).norm() / b.float().norm()).item()

    torch.manual_seed(12)
    m = Bottleneck(in_ch, ch, stride).cuda().to(memory_format=torch.channels_last)
    ref = Bottleneck(in_ch, ch, stride).cuda().to(memory_format=torch.channels_last)
    ref.load_state_dict(m.state_dict())
    m = m.to(torch.bfloat16)
    x = torch.randn(4, in_ch, 16, 16, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(ref(x.float()))

    def run(model, inp):
        xi = inp.clone().requires_grad_()
        y = model(xi)
        y.backward(g.to(y.dtype))
        out = (y.detach(), xi.grad, model.c1.conv.weight.grad)
        model.zero_grad(set_to_none=True)
        return out

    y32, gx32, gw32 = run(ref, x.float())
    yn, gxn, gwn = run(m, x)
    with monkeypatch.context() as mp:
        mp.setenv("TBAMD_FORCE_REFERENCE", "1")
        ya, gxa, gwa = run(m, x)
    assert rel(yn, y32) < 3e-2
    assert relnorm(gxn, gx32) <= 1.5 * relnorm(gxa, gx32) + 1e-2
    assert relnorm(gwn, gw32) <= 1.5 * relnorm(gwa, gw32) + 1e-2


def test_conv_bn_stats_fusion():
    from torchbooster_amd.models.resnet import ConvBNAct

    torch.manual_seed(6)
    m = ConvBNAct(64, 128, 3, 1).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref = ConvBNAct(64, 128, 3, 1).cuda().to(memory_format=torch.channels_last)
    ref.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in m.state_dict().items()})
    x = torch.randn(4, 64, 20, 20, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = m(x)
    with torch.no_grad():
        z = F.conv2d(x.float(), ref.conv.weight.float(), None, 1, 1)
        yr = F.relu(F.batch_norm(z, None, None, ref.bn.weight, ref.bn.bias, True, 0.1, 1e-5))
    assert rel(y, yr) < 2e-2
    rm = z.mean(dim=(0, 2, 3)) * 0.1
    assert torch.allclose(m.bn.running_mean, rm, atol=2e-3, rtol=2e-2)


def test_resnet50_bf16_step_runs_native():
    from torchbooster_amd import models, utils
    from torchbooster_amd.ops.loss import cross_entropy_accuracy
    from torchbooster_amd.ops.optim import FusedAdamW

    torch.manual_seed(7)
    m = models.resnet50().cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = FusedAdamW(m.parameters(), lr=1e-3)
    x = torch.randn(8, 3, 64, 64, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device=DEV)
    losses = []
    for _ in range(3):
        loss, acc = cross_entropy_accuracy(m(x), y, 0.1)
        utils.step(loss, opt, clip=1.0)
        losses.append(loss.item())
    assert all(l == l for l in losses) and losses[-1] < losses[0]


def test_device_normalize_matches_cpu():
    from torchbooster_amd.data import device_normalize

    torch.manual_seed(8)
    imgs = torch.randint(0, 256, (4, 10, 12, 3), dtype=torch.uint8)
    offs = torch.tensor([[0, 0], [1, 2], [-2, -1], [2, -2]], dtype=torch.int32)
    flip = torch.tensor([0, 1, 1, 0], dtype=torch.uint8)
    a = device_normalize(imgs.cuda(), (0.4, 0.5, 0.6), (0.2, 0.25, 0.3), (8, 9), offs, flip, torch.float32)
    b = device_normalize(imgs, (0.4, 0.5, 0.6), (0.2, 0.25, 0.3), (8, 9), offs, flip, torch.float32)
    assert torch.allclose(a.cpu(), b, atol=1e-5)


def test_pinned_prefetcher_from_lmdb(tmp_path):
    import numpy as np

    from torchbooster_amd.data import LMDBImageDataset, PinnedPrefetcher

    imgs = np.random.randint(0, 256, (37, 8, 8, 3), dtype=np.uint8)
    LMDBImageDataset.prepare(tmp_path, imgs, list(range(37)))
    ds = LMDBImageDataset(str(tmp_path))
    pf = PinnedPrefetcher(ds, 8, shuffle=False, mean=(0, 0, 0), std=(1, 1, 1), dtype=torch.float32)
    seen = []
    for x, y in pf:
        assert x.is_cuda and x.shape == (8, 3, 8, 8)
        seen.extend(y.tolist())
        i = y[0].item()
        assert torch.allclose(x[0].cpu(), torch.from_numpy(imgs[i]).permute(2, 0, 1).float() / 255, atol=1e-6)
    assert seen == list(range(32))


def test_zero_copy_grad_slots(monkeypatch):
    """After zero_grad(set_to_none) the conv / BN / linear backward kernels write
    straight into the optimizer's persistent grad store (no copy, no add), and
    the values equal the copy/accumulate path's."""
    from torchbooster_amd import models
    from torchbooster_amd.ops import conv as nconv
    from torchbooster_amd.ops.optim import FusedAdamW

    # deterministic kernels only (MIOpen's split-k conv grads use atomics)
    monkeypatch.setitem(nconv._FORCE, "fwd", "native")
    monkeypatch.setitem(nconv._FORCE, "dgrad", "native")
    monkeypatch.setitem(nconv._FORCE, "wgrad", "native")
    torch.manual_seed(3)
    m = models.resnet18(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = FusedAdamW(m.parameters(), lr=0.0, weight_decay=0.0)
    x = torch.randn(4, 3, 64, 64, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device=DEV)
    F.cross_entropy(m(x).float(), y).backward()
    opt.step()  # builds the grad store (slots)
    opt.zero_grad(set_to_none=False)  # bound, zeroed views: autograd adds into them
    F.cross_entropy(m(x).float(), y).backward()
    ref = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    opt.zero_grad(set_to_none=True)  # unbound: kernels write into the slots
    F.cross_entropy(m(x).float(), y).backward()
    in_slot = 0
    for n, p in m.named_parameters():
        assert p.grad is not None, n
        err = ((p.grad.float() - ref[n]).norm() / ref[n].norm().clamp_min(1e-12)).item()
        # the stride-2 input gradients are native (parity-class kernels) now: every
        # gradient is a deterministic function of its inputs except where split
        # reductions re-associate (bf16 rounding of the slot vs the fresh tensor)
        tol = 1e-3 if n.startswith(("fc.", "layer4.1.")) else 2e-2
        assert err < tol, (n, err)
        in_slot += int(p.grad.data_ptr() == p._tb_slot.data_ptr())
    n_params = len(list(m.parameters()))
    # every conv (except the 3-channel stem), BN and the classifier adopt their slot
    assert in_slot >= n_params - 1, (in_slot, n_params)


@pytest.mark.parametrize("kind", ["layernorm", "instancenorm"])
def test_norm_affine_grads_in_slots(kind):
    """LayerNorm / InstanceNorm (GroupNorm kernel) weight and bias gradients are written by the
    kernel's final reduction straight into the optimizer's grad store after
    zero_grad(set_to_none=True): same values as the bound/accumulate path, no per-step copy."""
    from torchbooster_amd.ops.norm import InstanceNormAct2d, LayerNorm
    from torchbooster_amd.ops.optim import FusedAdamW

    torch.manual_seed(5)
    if kind == "layernorm":
        m = LayerNorm(256).cuda()
        x = torch.randn(4, 37, 256, device=DEV).to(torch.bfloat16)
    else:
        m = InstanceNormAct2d(64, act="relu").cuda()
        x = torch.randn(2, 64, 24, 24, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.5, 0.5)
    g = torch.randn_like(x)
    opt = FusedAdamW(m.parameters(), lr=0.0, weight_decay=0.0)
    (m(x).float() * g.float()).sum().backward()
    opt.step()  # builds the grad store (slots)
    opt.zero_grad(set_to_none=False)
    (m(x).float() * g.float()).sum().backward()
    ref = {n: p.grad.clone() for n, p in m.named_parameters()}
    opt.zero_grad(set_to_none=True)
    (m(x).float() * g.float()).sum().backward()
    for n, p in m.named_parameters():
        assert p.grad.data_ptr() == p._tb_slot.data_ptr(), n
        torch.testing.assert_close(p.grad, ref[n], rtol=1e-5, atol=1e-5)
    # and against fp32 ATen
    w, b = (p.detach().clone().requires_grad_() for p in (m.weight, m.bias))
    xf = x.float()
    if kind == "layernorm":
        yf = F.layer_norm(xf, (256,), w, b, m.eps)
    else:
        yf = F.relu(F.instance_norm(xf, weight=w, bias=b, eps=m.eps))
    (yf * g.float()).sum().backward()
    for p, r in ((m.weight, w.grad), (m.bias, b.grad)):
        assert ((p.grad - r).norm() / r.norm()).item() < 2e-2


@pytest.mark.parametrize("N,C,H", [(4, 64, 32), (2, 64, 17), (3, 128, 9)])
def test_bn_relu_maxpool_fused(N, C, H):
    """Fused BN + ReLU + 3x3/2 max-pool (and its argmax-gather backward) vs fp32."""
    from torchbooster_amd.ops.norm import BatchNormAct2d

    torch.manual_seed(21)
    bn = BatchNormAct2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xa, xr = x.clone().requires_grad_(), x.float().requires_grad_()
    y = bn.forward_maxpool(xa, 3, 2, 1)
    w, b = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    yr = F.max_pool2d(F.relu(F.batch_norm(xr, None, None, w, b, True, 0.1, 1e-5)), 3, 2, 1)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert rel(y, yr) < 2e-2
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g)

    def relnorm(a, b_):
        return ((a.float() - b_.float()).norm() / b_.float().norm()).item()

    assert relnorm(xa.grad, xr.grad) < 3e-2
    assert relnorm(bn.weight.grad, w.grad) < 2e-2
    assert relnorm(bn.bias.grad, b.grad) < 2e-2
    assert int(bn.num_batches_tracked) == 1


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_bn_relu_maxpool_fused_backward_vs_unfused(monkeypatch, dt):
    """The stem backward with the pool-input gradient gathered inside the BN passes
    (csrc/pool_gather.h, bn_backward_pool) against the unfused gather kernel + BN backward and
    against fp32 PyTorch: the fused dz never rounds to the storage dtype, so it is at least as
    close to the reference."""
    from torchbooster_amd.ops import norm as NM

    torch.manual_seed(5)
    N, C, H = 3, 64, 30
    x = torch.randn(N, C, H, H, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
    g = torch.randn(N, C, 15, 15, device=DEV)
    w0, b0 = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    xr = x.detach().float().clone().requires_grad_()
    wr, br = w0.clone().requires_grad_(), b0.clone().requires_grad_()
    F.max_pool2d(F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5)), 3, 2, 1).backward(g)
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(NM, "_POOL_FUSED_BWD", fused)
        bn = NM.BatchNormAct2d(C).cuda()
        with torch.no_grad():
            bn.weight.copy_(w0)
            bn.bias.copy_(b0)
        xa = x.detach().clone().requires_grad_()
        bn.forward_maxpool(xa, 3, 2, 1).backward(g.to(dt))
        out[fused] = (xa.grad.float(), bn.weight.grad.float(), bn.bias.grad.float())

    def relnorm(a, b_):
        return ((a - b_).norm() / b_.norm()).item()

    for i, ref in enumerate((xr.grad, wr.grad, br.grad)):
        ef, eu = relnorm(out[True][i], ref), relnorm(out[False][i], ref)
        assert ef < (2e-2 if dt == torch.bfloat16 else 1e-4), (i, ef)
        assert ef <= eu * 1.1 + 1e-6, (i, ef, eu)


def test_residual_grad_link_matches_materialised(monkeypatch):
    """Identity Bottleneck: the masked residual-gradient hand-off (1-bit ReLU
    mask + dgrad epilogue) equals the materialised dres path."""
    from torchbooster_amd.models import resnet as R
    from torchbooster_amd.ops import conv as nconv

    for d in ("fwd", "dgrad", "wgrad"):
        monkeypatch.setitem(nconv._FORCE, d, "native")
    torch.manual_seed(14)
    m = R.Bottleneck(256, 64, 1).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    x = torch.randn(4, 256, 16, 16, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = torch.randn(4, 256, 16, 16, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def run():
        xi = x.clone().requires_grad_()
        y = m(xi)
        y.backward(g)
        out = [y.detach().clone(), xi.grad.clone()] + [p.grad.clone() for p in m.parameters()]
        m.zero_grad(set_to_none=True)
        return out

    linked = run()
    monkeypatch.setattr(R, "ResidualGradLink", lambda: None)
    plain = run()
    for a, b in zip(linked, plain):
        assert ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item() < 1e-2


def test_bn_backward_partials_from_dgrad_epilogue(monkeypatch):
    """ResNet-50 chain: BN backward partial sums emitted by the consumer conv's
    dgrad epilogue give the same gradients as the BN's own partial pass."""
    from torchbooster_amd.models import resnet as R
    from torchbooster_amd.ops import conv as nconv

    for d in ("fwd", "dgrad", "wgrad"):
        monkeypatch.setitem(nconv._FORCE, d, "native")
    torch.manual_seed(15)
    m = R.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
    x = torch.randn(4, 3, 64, 64, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device=DEV)

    def run():
        F.cross_entropy(m(x).float(), y).backward()
        out = {n: p.grad.float().clone() for n, p in m.named_parameters()}
        m.zero_grad(set_to_none=True)
        return out

    linked = run()
    monkeypatch.setattr(R, "BnBwdLink", lambda: None)
    plain = run()
    # fp32 reference of the same weights (ATen path): both bf16 variants are
    # judged by their distance to it, so summation-order noise amplified
    # through 50 BN backwards (tiny batch, near-cancelling bias grads) does not
    # read as a linking bug
    import copy

    m32 = copy.deepcopy(m).float()
    F.cross_entropy(m32(x.float()), y).backward()
    ref = {n: p.grad.float() for n, p in m32.named_parameters()}
    worse = {}
    for n in plain:
        if n.startswith("stem.conv"):
            continue  # MIOpen wgrad of the 3-channel stem (atomics)
        den = ref[n].norm().clamp_min(1e-12)
        e_link = ((linked[n] - ref[n]).norm() / den).item()
        e_plain = ((plain[n] - ref[n]).norm() / den).item()
        worse[n] = (e_link - 1.5 * e_plain, e_link, e_plain)
    bad = {n: v for n, v in worse.items() if v[0] > 2e-2}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:5]


@pytest.mark.parametrize("N,C,H,k,s,p", [(1, 64, 512, 2, 2, 0), (2, 128, 33, 2, 2, 0), (4, 64, 56, 3, 2, 1),
                                         (2, 512, 32, 2, 2, 0)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_native_maxpool_matches_aten(N, C, H, k, s, p, dt):
    from torchbooster_amd.ops.pool import max_pool2d

    x = torch.randn(N, C, H, H, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = max_pool2d(x, k, s, p)
    xf = x.detach().float().requires_grad_(True)
    yf = torch.nn.functional.max_pool2d(xf, k, s, p)
    assert y.shape == yf.shape and torch.equal(y.float(), yf)
    g = torch.randn_like(yf)
    y.backward(g.to(dt))
    yf.backward(g)
    if dt == torch.float32:  # no ties: the same tap wins
        assert torch.allclose(x.grad, xf.grad, atol=1e-6)
    else:  # bf16 windows hold ties (either tap is a valid argmax): every output grad lands once
        assert torch.allclose(x.grad.float().sum(), g.to(dt).float().sum(), rtol=1e-2, atol=1e-1)  # bf16 dx rounding
        hit = x.grad != 0
        assert torch.equal(torch.nn.functional.max_pool2d(x.detach().float(), k, s, p), yf.detach())
        assert hit.sum() <= yf.numel()


@pytest.mark.parametrize("N,H,K", [(2, 224, 64), (3, 37, 64), (1, 64, 128)])
def test_native_stem_conv_matches_fp32(N, H, K, monkeypatch):
    """7x7/2 stem on the native kernel (pre-padded 4-channel image, packed weights) vs fp32
    F.conv2d, plus its fused BN statistics; the weight gradient (MIOpen) flows."""
    from torchbooster_amd.ops import conv as convmod

    monkeypatch.setitem(convmod._FORCE, "fwd", "native")
    torch.manual_seed(H)
    x = torch.randn(N, 3, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, 3, 7, 7, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_(True)
    y, stats = convmod.conv_stem(x, w, True)
    ref = torch.nn.functional.conv2d(x.float(), w.detach().float(), None, 2, 3)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
    # stats: per-tile (sum, sum of squares) of the bf16 outputs
    tot = stats.double().sum(0)
    yb = y.double()
    assert torch.allclose(tot[0], yb.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    assert torch.allclose(tot[1], (yb * yb).sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    g = torch.randn_like(y, dtype=torch.float32)
    (y.float() * g).sum().backward()
    wf = w.detach().float().requires_grad_(True)
    (torch.nn.functional.conv2d(x.float(), wf, None, 2, 3) * g).sum().backward()
    monkeypatch.setitem(convmod._FORCE, "wgrad", "native")
    w2 = w.detach().clone().requires_grad_(True)
    y2, _ = convmod.conv_stem(x, w2, True)
    (y2.float() * g).sum().backward()
    for gw in (w.grad, w2.grad):  # first: autotuned route, second: the native weight-gradient kernel
        err = ((gw.float() - wf.grad).norm() / wf.grad.norm()).item()
        assert err < 2e-2, err


@pytest.mark.parametrize("N,C,H,K,R,pad", [(2, 128, 28, 128, 3, 1), (2, 256, 56, 512, 1, 0), (3, 64, 15, 128, 3, 1),
                                           (2, 64, 15, 64, 1, 0), (1, 128, 14, 256, 3, 1)])
def test_native_stride2_dgrad_matches_fp32(N, C, H, K, R, pad):
    """Stride-2 input gradient as four output-parity sub-convolutions on the native kernel."""
    from torchbooster_amd.ops import _ext

    torch.manual_seed(H + K)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    P = (H + 2 * pad - R) // 2 + 1
    dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    C_ = _ext.native()
    dx = C_.conv2d_dgrad_s2(dy, C_.conv_flip_weight(w), R, R, pad, H, H)[0]
    xf = x.float().requires_grad_(True)
    torch.nn.functional.conv2d(xf, w.float(), None, 2, pad).backward(dy.float())
    assert dx.shape == xf.grad.shape and dx.is_contiguous(memory_format=torch.channels_last)
    err = ((dx.float() - xf.grad).norm() / xf.grad.norm()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("N,C,H,K,R,st,pad", [(2, 64, 30, 128, 5, 2, 2), (2, 128, 28, 128, 7, 2, 3),
                                              (2, 128, 16, 64, 3, 3, 1), (3, 64, 19, 64, 5, 3, 2),
                                              (2, 64, 17, 128, 3, 2, 4), (1, 64, 12, 64, 8, 2, 3),
                                              (2, 128, 20, 64, 1, 3, 0), (2, 64, 23, 64, 7, 3, 0)])
def test_native_phase_dgrad_any_taps_stride3_matches_fp32(N, C, H, K, R, st, pad):
    """The phase-class input gradient generalised (csrc/conv.hip conv_dgrad_s2): stride 2 with up
    to 16 taps per class (5x5, 7x7, 8x8), stride 3 (9 classes), padding beyond R - 1, 1x1 / 3."""
    from torchbooster_amd.ops import _ext

    torch.manual_seed(H + K + R + st)
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") * (C * R * R) ** -0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    C_ = _ext.native()
    assert C_.conv_dgrad_s2_supported(R, R, st)
    dx = C_.conv2d_dgrad_s2(dy, C_.conv_flip_weight(w), R, R, pad, H, H, stride=st)[0]
    xf = x.float().requires_grad_(True)
    torch.nn.functional.conv2d(xf, w.float(), None, st, pad).backward(dy.float())
    assert dx.shape == xf.grad.shape and dx.is_contiguous(memory_format=torch.channels_last)
    err = ((dx.float() - xf.grad).norm() / xf.grad.norm()).item()
    assert err < 1e-2, err


def test_native_phase_dgrad_refuses_too_many_taps():
    from torchbooster_amd.ops import _ext

    C_ = _ext.native()
    assert not C_.conv_dgrad_s2_supported(9, 9, 2) and not C_.conv_dgrad_s2_supported(3, 3, 4)
    dy = torch.randn(1, 64, 4, 4, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = torch.randn(64, 64, 9, 9, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError, match="taps per phase class"):
        C_.conv2d_dgrad_s2(dy, wt, 9, 9, 4, 8, 8)


def test_native_stride2_dgrad_bn_partials():
    """Stride-2 dgrad with the BN-backward partial sums of the BN that produced the conv input
    (mode 1: ReLU mask recomputed from the BN input), rows of the four parity classes stacked."""
    from torchbooster_amd.ops import _ext

    torch.manual_seed(7)
    N, C, H, K, R, pad = 2, 128, 28, 128, 3, 1
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    P = (H + 2 * pad - R) // 2 + 1
    dy = torch.randn(N, K, P, P, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xb = torch.randn(N * H * H, C, device="cuda").to(torch.bfloat16)
    scale, shift, mean = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    C_ = _ext.native()
    wt = C_.conv_flip_weight(w)
    dx, part = C_.conv2d_dgrad_s2(dy, wt, R, R, pad, H, H, 1, xb, scale, shift, mean, None)
    dx0 = C_.conv2d_dgrad_s2(dy, wt, R, R, pad, H, H)[0]
    assert torch.equal(dx, dx0)
    rows = dx.permute(0, 2, 3, 1).reshape(-1, C).double()
    keep = (xb.float() * scale + shift) > 0
    dz = torch.where(keep, rows, torch.zeros_like(rows))
    tot = part.double().sum(0)
    assert torch.allclose(tot[0], dz.sum(0), rtol=1e-4, atol=1e-2)
    assert torch.allclose(tot[1], (dz * (xb.double() - mean.double())).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("N,C,H", [(256, 2048, 7), (4, 512, 1), (3, 72, 5)])
def test_global_avgpool_head(N, C, H):
    """K7: native NHWC global average pool (fwd + broadcast bwd) vs fp32 ATen."""
    from torchbooster_amd.models.resnet import _GlobalAvgPoolNHWC

    torch.manual_seed(N + C)
    x = torch.randn(N, C, H, H, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_()
    y = _GlobalAvgPoolNHWC.apply(xa)
    xr = x.float().requires_grad_()
    yr = xr.mean((2, 3))
    assert rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.to(y.dtype))
    yr.backward(g)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last) and rel(xa.grad, xr.grad) < 1e-2


def test_flip_cache_tables_keyed_by_shape():
    """_FlipCache launch tables are reused by signature; a later parameter can reuse a dead one's
    Python id and both device addresses, so the signature must carry the shape (a table built for
    a bigger weight flipped past the end of the new copy: a GPU fault seen in round 5)."""
    from torchbooster_amd.ops import conv as CV

    fc = CV._FlipCache()
    for K, C in ((128, 64), (64, 128)):
        p = torch.nn.Parameter(torch.randn(K, C, 3, 3, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last))
        wt = fc.get(p, p)
        ref = p.detach().flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        assert torch.equal(wt, ref)
    for sig in fc._tables:
        assert all(len(e) == 5 and isinstance(e[3], tuple) for e in sig), sig


def test_batchnorm_on_many_streams():
    """More streams than the finalize kernel has ticket rows (32): the later streams take the
    single-phase finalize instead of sharing arrival counters; every stream's result is exact."""
    from torchbooster_amd.ops.norm import batch_norm_act

    torch.manual_seed(7)
    C = 128
    x = (torch.randn(64, C, 28, 28, device=DEV) * 2 + 1).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)  # enough rows for the two-phase finalize
    w = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    ref = F.batch_norm(x.float(), None, None, w, b, True, 0.1, 1e-5).relu()
    streams = [torch.cuda.Stream() for _ in range(40)]
    outs = []
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
            outs.append(batch_norm_act(x, w, b, rm, rv, True, 0.1, 1e-5, None, "relu", 0.0))
    for s in streams:
        torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for y in outs:  # (two-phase and single-phase finalizes sum in different orders: not bitwise)
        assert rel(y, ref) < 2e-2
