"""Big-tile implicit-GEMM conv (csrc/conv_big.hip: 8 waves, one workgroup per CU, a ring of
direct-to-LDS stages, 16x16x32 or 32x32x16 MFMA) against plain PyTorch fp32 references, for every
instantiated tile configuration and every fused epilogue: bias / ReLU, BatchNorm statistics,
residual addend (plain and masked by saved ReLU bits), and the BN-backward partials of the dgrad
use (BNB 1 / 2 / 3).  Reference: the ResNet convs of examples/img_cls/resnet/resnet.py:44-68,111
(cuDNN there)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.ops._ext import native  # noqa: E402

CONFIGS = [(128, 256, 16, 2), (128, 256, 16, 3), (128, 256, 32, 3), (128, 128, 16, 4), (64, 256, 16, 3),
           (64, 256, 32, 3), (256, 256, 16, 2), (256, 128, 16, 3),
           (256, 256, 32, 2), (256, 128, 32, 3), (128, 128, 32, 4)]


def _cl(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.fixture
def big():
    C = native()
    old = C.conv_get_big()
    yield C
    C.conv_set_big(old)


def _bits_to_mask(bits, NPQ, K):
    # [NPQ, K/8] bytes, bit e of byte j = channel 8 j + e
    b = bits.long().reshape(NPQ, K // 8, 1)
    return ((b >> torch.arange(8, device=bits.device)) & 1).reshape(NPQ, K).bool()


@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("N,C,H,K,R,st,pad", [(2, 64, 20, 256, 3, 1, 1), (3, 128, 15, 256, 1, 1, 0),
                                              (2, 192, 14, 256, 3, 2, 1)])
def test_big_forward_stats(big, cfg, N, C, H, K, R, st, pad):
    bm, bn, mf, stg = cfg
    code = big.conv_big_encode(bm, bn, mf, stg)
    torch.manual_seed(C + H + K + R)
    x = _cl(torch.randn(N, C, H, H, device="cuda"))
    w = _cl(torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5)
    big.conv_set_big(code)
    assert big.conv_big_choice(N * ((H + 2 * pad - R) // st + 1) ** 2, C, K, R, R, st, pad) == code
    y, stats = big.conv2d_fwd(x, w, None, st, pad, False, True)
    ref = F.conv2d(x.float(), w.float(), stride=st, padding=pad)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    # statistics rows: one per pixel tile of bn pixels; their sum = the bf16 output's sums
    NPQ = y.shape[0] * y.shape[2] * y.shape[3]
    assert stats.shape == ((NPQ + bn - 1) // bn, 2, K)
    yf = y.permute(0, 2, 3, 1).reshape(-1, K).float()
    s = stats.double().sum(0)
    torch.testing.assert_close(s[0], yf.double().sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s[1], (yf.double() ** 2).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("cfg", [(128, 256, 16, 3), (128, 256, 32, 3), (64, 256, 16, 3), (256, 256, 16, 2)])
@pytest.mark.parametrize("bias,relu", [(True, False), (True, True), (False, True)])
def test_big_forward_bias_relu(big, cfg, bias, relu):
    bm, bn, mf, stg = cfg
    torch.manual_seed(1)
    x = _cl(torch.randn(2, 64, 18, 18, device="cuda"))
    w = _cl(torch.randn(256, 64, 3, 3, device="cuda") / 24.0)
    b = torch.randn(256, device="cuda") if bias else None
    big.conv_set_big(big.conv_big_encode(bm, bn, mf, stg))
    y = big.conv2d_fwd(x, w, b, 1, 1, relu, False)[0]
    ref = F.conv2d(x.float(), w.float(), b, padding=1)
    if relu:
        ref = F.relu(ref)
    err = (y.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("cfg", CONFIGS)
@pytest.mark.parametrize("bnb_mode,add", [(0, 1), (0, 2), (1, 0), (2, 0), (3, 0), (2, 2), (1, 1)])
def test_big_dgrad_epilogues(big, cfg, bnb_mode, add):
    """The input-gradient form: y = conv(dy, w) (+ addend, optionally masked) and the BN-backward
    partials (sum dz, sum dz (xb - mean)) with dz = y * act'(BN(xb)) of the BN in front."""
    bm, bn, mf, stg = cfg
    torch.manual_seed(bnb_mode * 10 + add)
    N, Kin, H, Kout = 2, 128, 17, 256  # dy has Kin channels; the output (dX) Kout
    dy = _cl(torch.randn(N, Kin, H, H, device="cuda"))
    w = _cl(torch.randn(Kout, Kin, 3, 3, device="cuda") / 34.0)
    NPQ = N * H * H
    kw = {}
    ref = F.conv2d(dy.float(), w.float(), padding=1)
    if add:
        addend = _cl(torch.randn(N, Kout, H, H, device="cuda"))
        kw["addend"] = addend
        a = addend.float()
        if add == 2:
            abits = torch.randint(0, 256, (NPQ, Kout // 8), device="cuda", dtype=torch.uint8)
            kw["addend_mask"] = abits
            m = _bits_to_mask(abits, NPQ, Kout).reshape(N, H, H, Kout).permute(0, 3, 1, 2)
            a = a * m
        ref = ref + a
    if bnb_mode:
        xb = _cl(torch.randn(N, Kout, H, H, device="cuda"))
        mean = torch.randn(Kout, device="cuda") * 0.1
        kw.update(bnb_mode=bnb_mode, bnb_x=xb, bnb_mean=mean)
        if bnb_mode == 1:
            scale = torch.rand(Kout, device="cuda") + 0.5
            shift = torch.randn(Kout, device="cuda") * 0.2
            kw.update(bnb_scale=scale, bnb_shift=shift)
        if bnb_mode == 2:
            bits = torch.randint(0, 256, (NPQ, Kout // 8), device="cuda", dtype=torch.uint8)
            kw["bnb_bits"] = bits
    big.conv_set_big(big.conv_big_encode(bm, bn, mf, stg))
    outs = big.conv2d_fwd(dy, w, None, 1, 1, False, False, **kw)
    y = outs[0]
    err = (y.float() - ref).abs().max().item()
    assert err <= 1.5e-2 * ref.abs().max().item(), err
    if bnb_mode:
        part = outs[1]
        assert part.shape == ((NPQ + bn - 1) // bn, 2, Kout)
        yv = y.permute(0, 2, 3, 1).reshape(NPQ, Kout).float().double()
        xv = xb.permute(0, 2, 3, 1).reshape(NPQ, Kout).float().double()
        if bnb_mode == 1:
            keep = (xv * scale.double() + shift.double()) > 0
        elif bnb_mode == 2:
            keep = _bits_to_mask(bits, NPQ, Kout)
        else:
            keep = torch.ones_like(yv, dtype=torch.bool)
        dz = torch.where(keep, yv, torch.zeros_like(yv))
        p = part.double().sum(0)
        torch.testing.assert_close(p[0], dz.sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(p[1], (dz * (xv - mean.double())).sum(0), rtol=1e-4, atol=1e-2)


def test_big_tail_and_odd_shapes(big):
    """Pixel counts that are not a multiple of the tile (rows past NPQ read the zero page and are
    never stored), more channel tiles than pixel tiles, stride 2 with padding."""
    torch.manual_seed(3)
    for (N, C, H, K, R, st, pad) in [(1, 64, 5, 512, 3, 2, 1), (1, 320, 7, 128, 1, 1, 0), (5, 64, 9, 64, 3, 1, 1)]:
        x = _cl(torch.randn(N, C, H, H, device="cuda"))
        w = _cl(torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5)
        ref = F.conv2d(x.float(), w.float(), stride=st, padding=pad)
        for cfg in CONFIGS:
            if K % cfg[0]:
                continue
            big.conv_set_big(big.conv_big_encode(*cfg))
            y, stats = big.conv2d_fwd(x, w, None, st, pad, False, True)
            err = (y.float() - ref).abs().max().item()
            assert err <= 1e-2 * ref.abs().max().item(), (cfg, err)
            yf = y.permute(0, 2, 3, 1).reshape(-1, K).float().double()
            torch.testing.assert_close(stats.double().sum(0)[0], yf.sum(0), rtol=1e-4, atol=1e-2)


def test_big_heuristic_route_and_training_step(big):
    """TBAMD_CONV_BIG=1 (the heuristic) inside a ResNet-50 training step: every conv2d_fwd call of
    the step (forward with BN statistics, input-gradient forms with the residual addend and the
    BN-backward partials) is recomputed in context, on the same tensors, with the 128x128 kernels.
    The big tiles reduce over k in the same order, so the outputs must be bitwise equal; the
    statistics / partials rows are summed over a different pixel tiling, so their totals agree to
    rounding.  (An end-to-end gradient comparison is not a usable bar: a random-init 53-BN network
    amplifies a 1e-8 change in statistics summation order into O(1) gradient differences -- see
    profiles/r05_big/README.md.)"""
    from torchbooster_amd import models

    orig = big.conv2d_fwd
    calls = []

    def patched(*a, **k):
        out = orig(*a, **k)
        mode = big.conv_get_big()
        big.conv_set_big(0)
        ref = orig(*a, **k)
        big.conv_set_big(mode)
        ydiff = (out[0].float() - ref[0].float()).abs().max().item()
        adiff = 0.0
        if len(out) > 1 and out[1] is not None and out[1].dim() == 3:
            s1, s0 = out[1].double().sum(0), ref[1].double().sum(0)
            adiff = ((s1 - s0).abs().max() / s0.abs().max().clamp_min(1e-30)).item()
        calls.append((tuple(a[0].shape), tuple(a[1].shape), ydiff, adiff))
        return out

    big.conv2d_fwd = patched
    try:
        big.conv_set_big(1)
        torch.manual_seed(0)
        m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).to(torch.bfloat16)
        x = torch.randn(8, 3, 96, 96, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        m(x).float().square().mean().backward()
        torch.cuda.synchronize()
    finally:
        big.conv2d_fwd = orig
    assert len(calls) >= 60, len(calls)  # 52 forward convs (stem aside) + the input-gradient calls
    bad = [c for c in calls if c[2] != 0.0 or c[3] > 1e-5]
    assert not bad, bad[:8]
