"""Multi-process data-parallel runtime on CPU (gloo, world_size 2/4).

Covers: launch/job spawn path, rank helpers, local groups, the native bucketed
reducer (grad equality vs a single-process reference, GAN-style interleaved
forwards — SURVEY.md A.2 B10, accumulation via no_sync / utils.step), buffer
broadcast and param broadcast at wrap time.
"""
import os
import tempfile

import pytest
import torch
import torch.nn as nn

import torchbooster_amd.distributed as dist
from torchbooster_amd import utils
from torchbooster_amd.parallel import DistributedDataParallel


def _save(path, obj):
    torch.save(obj, path)


def _rank_helpers(out_dir):
    import torch.distributed as td

    r = dist.get_rank()
    info = {"rank": r, "world": dist.get_world_size(), "local": dist.get_local_rank(), "primary": dist.is_primary(),
            "backend": dist.backend()}
    t = torch.tensor([float(r)])
    lst = [torch.zeros(1) for _ in range(dist.get_world_size())] if dist.is_primary() else None
    dist.gather(t, lst)
    if dist.is_primary():
        info["gathered"] = [x.item() for x in lst]
    dist.synchronize()
    _save(os.path.join(out_dir, f"r{r}.pt"), info)


def test_launch_gloo_world2(tmp_path):
    dist.launch(_rank_helpers, 0, n_proc=2, args=(str(tmp_path),))
    a = torch.load(tmp_path / "r0.pt")
    b = torch.load(tmp_path / "r1.pt")
    assert a["world"] == 2 and b["rank"] == 1 and a["primary"] and not b["primary"]
    assert a["backend"] == "gloo"
    assert a["gathered"] == [0.0, 1.0]
    assert b["local"] == 1


def _multi_machine(out_dir):
    r = dist.get_rank()
    _save(os.path.join(out_dir, f"m{r}.pt"), {"rank": r, "local": dist.get_local_rank()})


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(8, 32), nn.GELU(), nn.BatchNorm1d(32), nn.Linear(32, 3))


def _ddp_equivalence(out_dir, bucket_mb):
    torch.manual_seed(100 + dist.get_rank())  # different init per rank: wrap must broadcast
    net = nn.Sequential(nn.Linear(8, 32), nn.GELU(), nn.BatchNorm1d(32), nn.Linear(32, 3))
    model = DistributedDataParallel(net, bucket_cap_mb=bucket_mb, first_bucket_mb=bucket_mb / 4)
    torch.manual_seed(7)
    x = torch.randn(16, 8)
    y = torch.randint(0, 3, (16,))
    r, w = dist.get_rank(), dist.get_world_size()
    xs, ys = x.chunk(w)[r], y.chunk(w)[r]
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for _ in range(3):
        loss = nn.functional.cross_entropy(model(xs), ys)
        utils.step(loss, opt)
    _save(os.path.join(out_dir, f"p{r}.pt"), {k: v.detach().clone() for k, v in net.state_dict().items()}
          | {"nb": model.num_buckets})


@pytest.mark.parametrize("bucket_mb", [0.0005, 32.0])
def test_ddp_grads_match_single_process(tmp_path, bucket_mb):
    dist.launch(_ddp_equivalence, 0, n_proc=2, args=(str(tmp_path), bucket_mb))
    p0 = torch.load(tmp_path / "p0.pt")
    p1 = torch.load(tmp_path / "p1.pt")
    for k in p0:
        # buffers are synced at the START of each forward (DDP semantics), so
        # after the last local forward they legitimately differ per rank
        if k == "nb" or "running" in k or "num_batches" in k:
            continue
        assert torch.allclose(p0[k].float(), p1[k].float(), atol=1e-6), k  # rank-identical
    if bucket_mb < 0.01:
        assert p0["nb"] > 2  # many small buckets exercised


def _manual_reference(out_dir):
    # emulate 2 ranks in one process: average the per-shard grads
    torch.manual_seed(100)
    net = nn.Sequential(nn.Linear(8, 32), nn.GELU(), nn.Linear(32, 3))
    torch.manual_seed(7)
    x = torch.randn(16, 8)
    y = torch.randint(0, 3, (16,))
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    for _ in range(3):
        opt.zero_grad()
        for xs, ys in zip(x.chunk(2), y.chunk(2)):
            (nn.functional.cross_entropy(net(xs), ys) / 2).backward()
        opt.step()
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def _ddp_vs_manual(out_dir):
    torch.manual_seed(100 + 0)  # rank 0 init is broadcast
    net = nn.Sequential(nn.Linear(8, 32), nn.GELU(), nn.Linear(32, 3))
    if dist.get_rank() == 1:
        for p in net.parameters():
            p.data.add_(1.0)  # garbage on rank 1, must be overwritten by the broadcast
    model = DistributedDataParallel(net, bucket_cap_mb=0.001, first_bucket_mb=0.0005)
    torch.manual_seed(7)
    x = torch.randn(16, 8)
    y = torch.randint(0, 3, (16,))
    r = dist.get_rank()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for _ in range(3):
        loss = nn.functional.cross_entropy(model(x.chunk(2)[r]), y.chunk(2)[r])
        utils.step(loss, opt)
    _save(os.path.join(out_dir, f"q{r}.pt"), {k: v.detach().clone() for k, v in net.state_dict().items()})


def test_ddp_matches_manual_average(tmp_path):
    dist.launch(_ddp_vs_manual, 0, n_proc=2, args=(str(tmp_path),))
    ref = _manual_reference(str(tmp_path))
    for r in (0, 1):
        got = torch.load(tmp_path / f"q{r}.pt")
        for k in ref:
            assert torch.allclose(got[k], ref[k], atol=1e-5), (r, k)


def _gan_ordering(out_dir):
    """Reference GAN loop order (gan.py:102-113): two D forwards before two
    backwards, plus a double-backward gradient penalty."""
    r = dist.get_rank()
    torch.manual_seed(0)
    G = DistributedDataParallel(nn.Sequential(nn.Linear(4, 16), nn.GELU(), nn.Linear(16, 6)))
    D = DistributedDataParallel(nn.Sequential(nn.Linear(6, 16), nn.GELU(), nn.Linear(16, 1)))
    og = torch.optim.AdamW(G.parameters(), lr=1e-2)
    od = torch.optim.AdamW(D.parameters(), lr=1e-2)
    torch.manual_seed(10 + r)
    for _ in range(2):
        real = torch.randn(8, 6)
        z = torch.randn(8, 4)
        fake = G(z)
        g_loss = torch.relu(1.0 - D(fake)).mean()
        fake = fake.detach()
        d_loss = torch.relu(1.0 - D(real)).mean() + torch.relu(1.0 + D(fake)).mean()
        alpha = torch.rand(8, 1)
        t = (alpha * real + (1 - alpha) * fake).requires_grad_(True)
        dt = D(t)
        gr = torch.autograd.grad(dt, t, torch.ones_like(dt), create_graph=True, retain_graph=True)[0]
        d_loss = d_loss + 5.0 * ((gr.norm(2, dim=1) - 1) ** 2).mean()
        utils.step(g_loss, og)
        utils.step(d_loss, od)
    _save(os.path.join(out_dir, f"g{r}.pt"), {
        "G": [p.detach().clone() for p in G.parameters()],
        "D": [p.detach().clone() for p in D.parameters()],
    })


def test_gan_ordering_stays_in_sync(tmp_path):  # B10
    dist.launch(_gan_ordering, 0, n_proc=2, args=(str(tmp_path),))
    a = torch.load(tmp_path / "g0.pt")
    b = torch.load(tmp_path / "g1.pt")
    for k in ("G", "D"):
        for x, y in zip(a[k], b[k]):
            assert torch.allclose(x, y, atol=1e-6), k


def _accum(out_dir):
    r = dist.get_rank()
    torch.manual_seed(0)
    net = nn.Linear(4, 2)
    model = DistributedDataParallel(net)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    torch.manual_seed(5 + r)
    xs = [torch.randn(3, 4) for _ in range(3)]
    for i, x in enumerate(xs):
        utils.step(model(x).pow(2).mean(), opt, accumulate=i < 2)
    _save(os.path.join(out_dir, f"a{r}.pt"), [p.detach().clone() for p in net.parameters()])


def test_accumulation_under_ddp(tmp_path):
    dist.launch(_accum, 0, n_proc=2, args=(str(tmp_path),))
    a = torch.load(tmp_path / "a0.pt")
    b = torch.load(tmp_path / "a1.pt")
    # manual: sum of 3 micro-batch grads per rank, averaged over ranks
    torch.manual_seed(0)
    net = nn.Linear(4, 2)
    grads = [torch.zeros_like(p) for p in net.parameters()]
    for r in range(2):
        torch.manual_seed(5 + r)
        xs = [torch.randn(3, 4) for _ in range(3)]
        for x in xs:
            net.zero_grad()
            net(x).pow(2).mean().backward()
            for g, p in zip(grads, net.parameters()):
                g += p.grad / 2
    with torch.no_grad():
        ref = [p - 0.1 * g for p, g in zip(net.parameters(), grads)]
    for x, y, z in zip(a, b, ref):
        assert torch.allclose(x, y, atol=1e-6)
        assert torch.allclose(x, z, atol=1e-5)


def _buffers(out_dir):
    r = dist.get_rank()
    bn = nn.BatchNorm1d(4)
    with torch.no_grad():
        bn.running_mean.fill_(float(r + 1))
    model = DistributedDataParallel(bn)
    rm_after_wrap = bn.running_mean.clone()
    model.train()
    model(torch.randn(5, 4) + 10 * r)  # forward broadcasts rank-0 buffers first
    _save(os.path.join(out_dir, f"b{r}.pt"), {"wrap": rm_after_wrap, "nbt": bn.num_batches_tracked.clone()})


def test_buffer_broadcast(tmp_path):
    dist.launch(_buffers, 0, n_proc=2, args=(str(tmp_path),))
    a = torch.load(tmp_path / "b0.pt")
    b = torch.load(tmp_path / "b1.pt")
    assert torch.equal(a["wrap"], b["wrap"]) and a["wrap"][0].item() == 1.0


def test_multi_machine_emulation(tmp_path):
    """n_machine=2 x 2 procs on one host: two launches share one tcp:// url."""
    import multiprocessing as mp

    url = f"tcp://127.0.0.1:{dist.find_free_port()}"
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=dist.launch, args=(_multi_machine, 0),
                         kwargs=dict(n_machine=2, machine_rank=m, dist_url=url, args=(str(tmp_path),), n_proc=2))
             for m in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = sorted((torch.load(tmp_path / f"m{r}.pt")["rank"], torch.load(tmp_path / f"m{r}.pt")["local"])
                 for r in range(4))
    assert got == [(0, 0), (1, 1), (2, 0), (3, 1)]


def test_sampler_and_sharding():
    from torchbooster_amd.config import DistributedIterableSizeableDataset

    shards = [list(DistributedIterableSizeableDataset(range(10), r, 3, 10)) for r in range(3)]
    flat = sorted(sum(shards, []))
    assert flat == list(range(10))
    assert all(len(set(a) & set(b)) == 0 for i, a in enumerate(shards) for b in shards[i + 1:])


def _desync_check(out_dir):
    r = dist.get_rank()
    torch.manual_seed(0)
    net = nn.Linear(4, 2)
    model = DistributedDataParallel(net, check_sync=True)  # verifies after every reduction
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    torch.manual_seed(5 + r)
    for _ in range(2):
        utils.step(model(torch.randn(3, 4)).pow(2).mean(), opt)
    # corrupt one rank's reduced grads: the self-check must catch it on every rank
    with torch.no_grad():
        if r == 1:
            model.parts[0].add_(1.0)
    caught = False
    try:
        model.verify_grad_sync()
    except RuntimeError as e:
        caught = "desync" in str(e)
    _save(os.path.join(out_dir, f"d{r}.pt"), {"caught": caught})


def test_ddp_desync_self_check(tmp_path):
    dist.launch(_desync_check, 0, n_proc=2, args=(str(tmp_path),))
    assert torch.load(tmp_path / "d0.pt")["caught"] and torch.load(tmp_path / "d1.pt")["caught"]


def _faulty(out_dir):
    net = DistributedDataParallel(nn.Linear(4, 2))
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    for _ in range(5):
        utils.step(net(torch.randn(3, 4)).sum(), opt)
    _save(os.path.join(out_dir, f"f{dist.get_rank()}.pt"), {"done": True})


def test_fault_injection_fails_fast(tmp_path, monkeypatch):
    """TORCHBOOSTER_FAULT_INJECT=1:3 raises on rank 1 at step 3; launch surfaces it."""
    from torchbooster_amd.fault import parse_spec

    assert parse_spec("1:3") == (1, 3, "raise") and parse_spec("0:2:exit") == (0, 2, "exit")
    monkeypatch.setenv("TORCHBOOSTER_FAULT_INJECT", "1:3")
    with pytest.raises(Exception, match="injected fault"):
        dist.launch(_faulty, 0, n_proc=2, args=(str(tmp_path),))
    assert not (tmp_path / "f1.pt").exists()


# --------------------------------------------------------------- round 2 additions
class _Mixed(nn.Module):
    """f32 and bf16 parameters in one model (separate per-dtype buckets), plus
    one branch that only some steps use."""

    def __init__(self):
        super().__init__()
        self.a = nn.Linear(8, 16)
        self.b = nn.Linear(16, 16).to(torch.bfloat16)
        self.c = nn.Linear(16, 3)
        self.never = nn.Linear(3, 3)  # used by no rank

    def forward(self, x):
        h = torch.relu(self.a(x))
        h = torch.relu(self.b(h.to(torch.bfloat16))).float()
        return self.c(h)


def _mixed_world(out_dir, reduce_dtype, find_unused):
    r, w = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(100 + r)  # rank-dependent init: the wrap must broadcast rank 0's
    net = _Mixed()
    model = DistributedDataParallel(net, bucket_cap_mb=0.001, first_bucket_mb=0.0005,
                                    reduce_dtype=reduce_dtype, find_unused_parameters=find_unused)
    torch.manual_seed(7)
    x = torch.randn(32, 8)
    y = torch.randint(0, 3, (32,))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for _ in range(2):
        utils.step(nn.functional.cross_entropy(model(x.chunk(w)[r]), y.chunk(w)[r]), opt)
    _save(os.path.join(out_dir, f"x{r}.pt"), {
        "params": {k: v.detach().float().clone() for k, v in net.state_dict().items()},
        "dtypes": sorted({str(b.dtype) for b in model.parts}),
        "never_grad_none": net.never.weight.grad is None,
        "rdt": [None if t is None else str(t.dtype) for t in model._rbufs],
    })


@pytest.mark.parametrize("reduce_dtype,find_unused", [(None, False), (torch.float32, True)])
def test_ddp_world4_mixed_dtype_buckets(tmp_path, reduce_dtype, find_unused):
    dist.launch(_mixed_world, 0, n_proc=4, args=(str(tmp_path), reduce_dtype, find_unused))
    outs = [torch.load(tmp_path / f"x{r}.pt") for r in range(4)]
    assert outs[0]["dtypes"] == ["torch.bfloat16", "torch.float32"]
    for o in outs[1:]:
        for k, v in outs[0]["params"].items():
            assert torch.allclose(v, o["params"][k], atol=1e-6), k  # rank-identical
    if reduce_dtype is not None:
        assert "torch.float32" in outs[0]["rdt"]  # the bf16 buckets reduce through f32 shadows
    # a parameter no rank used: None with find_unused_parameters (torch semantics),
    # zero-filled and reduced otherwise
    assert all(o["never_grad_none"] == find_unused for o in outs)


def _accum_world4(out_dir):
    r = dist.get_rank()
    torch.manual_seed(0)
    net = nn.Linear(4, 2)
    model = DistributedDataParallel(net)
    launched = []
    orig = model._launch
    model._launch = lambda b: (launched.append(b), orig(b))[1]
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    torch.manual_seed(5 + r)
    xs = [torch.randn(3, 4) for _ in range(4)]
    for i, x in enumerate(xs):
        utils.step(model(x).pow(2).mean(), opt, accumulate=i < 3)
    _save(os.path.join(out_dir, f"w{r}.pt"), {"p": [p.detach().clone() for p in net.parameters()],
                                              "launched": len(launched), "nb": model.num_buckets})


def test_accumulation_reduces_once_world4(tmp_path):
    """accumulate=True micro-steps run under no_sync_all: only the last backward
    all-reduces (once per bucket), and the result is the rank average of the sums."""
    dist.launch(_accum_world4, 0, n_proc=4, args=(str(tmp_path),))
    outs = [torch.load(tmp_path / f"w{r}.pt") for r in range(4)]
    assert all(o["launched"] == o["nb"] for o in outs)
    torch.manual_seed(0)
    net = nn.Linear(4, 2)
    grads = [torch.zeros_like(p) for p in net.parameters()]
    for r in range(4):
        torch.manual_seed(5 + r)
        for x in [torch.randn(3, 4) for _ in range(4)]:
            net.zero_grad()
            net(x).pow(2).mean().backward()
            for g, p in zip(grads, net.parameters()):
                g += p.grad / 4
    with torch.no_grad():
        ref = [p - 0.1 * g for p, g in zip(net.parameters(), grads)]
    for o in outs:
        for x, z in zip(o["p"], ref):
            assert torch.allclose(x, z, atol=1e-5)


def _forced_single(out_dir):
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(4, 8), nn.GELU(), nn.Linear(8, 2))
    model = DistributedDataParallel(net, force_reduce=True, bucket_cap_mb=0.0001, first_bucket_mb=0.0001)
    launched = []
    orig = model._launch
    model._launch = lambda b: (launched.append(b), orig(b))[1]
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    x = torch.randn(5, 4)
    utils.step(model(x).pow(2).mean(), opt)
    _save(os.path.join(out_dir, "f.pt"), {"launched": launched, "nb": model.num_buckets,
                                          "p": [p.detach().clone() for p in net.parameters()]})


def test_force_reduce_runs_collectives_on_one_rank(tmp_path):
    import torch.distributed as td

    td.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{dist.find_free_port()}", world_size=1, rank=0)
    try:
        _forced_single(str(tmp_path))
    finally:
        td.destroy_process_group()
    o = torch.load(tmp_path / "f.pt")
    assert o["nb"] > 1 and sorted(o["launched"]) == list(range(o["nb"]))  # every bucket, in order
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(4, 8), nn.GELU(), nn.Linear(8, 2))
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    x = torch.randn(5, 4)
    opt.zero_grad()
    net(x).pow(2).mean().backward()
    opt.step()
    for a, b in zip(o["p"], net.parameters()):
        assert torch.allclose(a, b, atol=1e-6)


def test_gradient_slot_is_taken_once_per_backward():
    """A parameter used by two nodes of one graph: the first node's kernel gets
    the zero-copy slot, the second a fresh tensor; autograd's sum is correct and
    the slot is released after AccumulateGrad (slot reuse)."""
    from torchbooster_amd.ops._ext import slot_alias, take_slot

    class _Mul(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(x)
            ctx.w = w
            return x * w

        @staticmethod
        def backward(ctx, dy):
            (x,) = ctx.saved_tensors
            s = take_slot(ctx.w)
            g = (dy * x).sum(0)
            if s is not None:
                s.copy_(g)
                return dy * ctx.w, slot_alias(s)
            return dy * ctx.w, g

    w = nn.Parameter(torch.ones(3))
    w._tb_slot = torch.zeros(3)
    x1, x2 = torch.full((2, 3), 2.0), torch.full((2, 3), 5.0)
    (_Mul.apply(x1, w).sum() + _Mul.apply(x2, w).sum()).backward()
    assert torch.allclose(w.grad, torch.full((3,), 14.0))  # 2*2 + 2*5, not 2x one of them
    assert not w._tb_slot_taken  # released by the post-accumulate hook
    w.grad = None
    _Mul.apply(x1, w).sum().backward()
    assert w.grad.data_ptr() == w._tb_slot.data_ptr()  # single use: zero-copy slot adopted


def test_shard_indices_match_distributed_sampler():
    """the device loaders shard like DistributedSampler (equal counts per
    rank, padded by wrapping unless drop_last), so no rank runs short of batches."""
    import numpy as np
    from torch.utils.data import DistributedSampler

    from torchbooster_amd.data import shard_indices

    for n in (10, 11, 12, 2):
        for drop_last in (False, True):
            ref = [list(DistributedSampler(range(n), num_replicas=3, rank=r, shuffle=False, drop_last=drop_last))
                   for r in range(3)]
            got = [shard_indices(np.arange(n), r, 3, drop_last).tolist() for r in range(3)]
            assert got == ref, (n, drop_last)
            assert len({len(g) for g in got}) == 1


def _gan_world2(out_dir):
    """GAN step order of examples/img_gen/dcgan (D step, then G step with D frozen)."""
    r = dist.get_rank()
    torch.manual_seed(0)
    G = DistributedDataParallel(nn.Sequential(nn.Linear(4, 16), nn.GELU(), nn.Linear(16, 8)))
    D = DistributedDataParallel(nn.Sequential(nn.Linear(8, 16), nn.GELU(), nn.Linear(16, 1)))
    counts = {"G": 0, "D": 0}
    for name, m in (("G", G), ("D", D)):
        orig = m._launch
        m._launch = (lambda o, n: lambda b: (counts.__setitem__(n, counts[n] + 1), o(b))[1])(orig, name)
    og, od = torch.optim.SGD(G.parameters(), lr=0.1), torch.optim.SGD(D.parameters(), lr=0.1)
    torch.manual_seed(10 + r)
    iters = 3
    for _ in range(iters):
        x = torch.randn(6, 8)
        fake = G(torch.randn(6, 4))
        d_loss = nn.functional.softplus(-D(x)).mean() + nn.functional.softplus(D(fake.detach())).mean()
        utils.step(d_loss, od)
        with utils.frozen(D):
            g_loss = nn.functional.softplus(-D(fake)).mean()
        utils.step(g_loss, og)
        assert all(p.requires_grad for p in D.parameters())
    _save(os.path.join(out_dir, f"g{r}.pt"), {"counts": counts, "nbG": G.num_buckets, "nbD": D.num_buckets,
                                              "D": [p.detach().clone() for p in D.parameters()],
                                              "G": [p.detach().clone() for p in G.parameters()]})


def test_gan_g_step_does_not_reduce_discriminator(tmp_path):
    """the generator step must not all-reduce D's gradient: exactly one
    D reduction (its buckets once) and one G reduction per iteration; grads stay rank-identical."""
    dist.launch(_gan_world2, 0, n_proc=2, args=(str(tmp_path),))
    o0, o1 = (torch.load(tmp_path / f"g{r}.pt") for r in range(2))
    for o in (o0, o1):
        assert o["counts"]["D"] == 3 * o["nbD"] and o["counts"]["G"] == 3 * o["nbG"]
    for a, b in zip(o0["D"] + o0["G"], o1["D"] + o1["G"]):
        assert torch.allclose(a, b, atol=1e-6)


def test_rccl_options_carry_the_pg_timeout(monkeypatch):
    """the RCCL Options object carries the job's PG timeout, so torch's
    init (which overrides the options with the timeout kwarg) no longer warns about a mismatch."""
    import datetime

    from torchbooster_amd import distributed as d

    opts = d._pg_options("nccl")
    if opts is None:
        pytest.skip("torch built without NCCL/RCCL")
    assert opts._timeout == d._DEFAULT_TIMEOUT
    assert opts.is_high_priority_stream
    assert d._DEFAULT_TIMEOUT == datetime.timedelta(minutes=int(__import__("os").environ.get("TBAMD_PG_TIMEOUT_MIN", "30")))
    assert d._pg_options("gloo") is None


def test_bucket_plan_tail_bucket_resnet50():
    """the first layers' gradients (the last ones ready) close in a bucket of
    their own of <= 1 MiB, so only that latency-bound collective is left after the final weight
    gradient; the C++ planner and its Python mirror agree."""
    import torch

    from torchbooster_amd import models
    from torchbooster_amd.ops._ext import DTYPE_CODE, available
    from torchbooster_amd.parallel import ddp as D

    m = models.resnet50(num_classes=1000)
    ps = [p for p in m.parameters()]
    numels = [p.numel() for p in ps]
    dts = [DTYPE_CODE[torch.bfloat16] if p.dim() == 4 else DTYPE_CODE[torch.float32] for p in ps]
    esz = [2 if p.dim() == 4 else 4 for p in ps]
    order = list(reversed(range(len(ps))))
    mib = 2 ** 20
    saved = D.available
    try:
        D.available = lambda: False
        py = D._plan(numels, dts, esz, order, 16 * mib, mib, mib)
    finally:
        D.available = saved
    if available():
        nat = D._plan(numels, dts, esz, order, 16 * mib, mib, mib)
        assert nat == py
    last = py["bucket_params"][-1]
    assert 0 in last  # the stem conv weight
    assert py["bucket_bytes"][-1] <= mib
    assert all(b >= mib for b in py["bucket_bytes"][:-1]), py["bucket_bytes"]
    # without the tail cap the last bucket is the multi-MiB tail of a regular bucket
    saved = D.available
    try:
        D.available = lambda: False
        old = D._plan(numels, dts, esz, order, 16 * mib, mib, 0)
    finally:
        D.available = saved
    assert old["bucket_bytes"][-1] > mib


# --------------------------------------------------------------- round 5 additions
def _probe_world(out_dir):
    os.environ["TBAMD_DDP_PRECISION_PROBE"] = "1"
    r, w = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(64, 256), nn.GELU(), nn.Linear(256, 64)).to(torch.bfloat16)
    model = DistributedDataParallel(net, bucket_cap_mb=0.05, first_bucket_mb=0.01)
    torch.manual_seed(11 + r)
    x = torch.randn(16, 64, dtype=torch.bfloat16)
    model(x).float().square().mean().backward()
    _save(os.path.join(out_dir, f"p{r}.pt"), {"summary": model.precision_summary(), "nb": model.num_buckets})


def test_ddp_precision_probe_world4(tmp_path):
    """the reducer can measure what reducing bf16 buckets in bf16 costs against
    an f32 reduction of the same local gradients (every bucket probed, every rank agrees)."""
    dist.launch(_probe_world, 0, n_proc=4, args=(str(tmp_path),))
    outs = [torch.load(tmp_path / f"p{r}.pt") for r in range(4)]
    s = outs[0]["summary"]
    assert s["buckets"] == outs[0]["nb"] and s["world"] == 4
    # bf16 result vs the f32 sum: at least the one final rounding, at most a few bf16 ulps
    assert 0.0 < s["round_rel_l2"] <= s["rel_l2"] < 2e-2, s
    for o in outs[1:]:
        assert o["summary"] == s  # the reduced buckets are rank-identical, so are their deviations


def _oneshot_partial_failure(out_dir):
    """OneShotAllReduce construction where only rank 1's staging allocation fails: every rank must
    raise (so the DDP fallback to RCCL is rank-consistent), nobody may block in a collective."""
    from torchbooster_amd.parallel import oneshot as OS

    r = dist.get_rank()

    class _Comm:
        def __init__(self, rank, *a):
            if rank == 1:
                raise RuntimeError("hipMalloc: out of memory")

        def handles(self):
            return b"h"

        def open(self, blobs):
            pass

    class _Native:
        OneShotComm = _Comm

    OS.native = lambda: _Native()
    try:
        OS.OneShotAllReduce(capacity_mb=1.0)
        got = "constructed"
    except RuntimeError as e:
        got = "raised:" + ("rank(s) 1" in str(e) and "setup" in str(e)).__str__()
    _save(os.path.join(out_dir, f"o{r}.pt"), {"got": got})


def test_oneshot_setup_failure_is_collective(tmp_path):
    dist.launch(_oneshot_partial_failure, 0, n_proc=2, args=(str(tmp_path),))
    assert [torch.load(tmp_path / f"o{r}.pt")["got"] for r in range(2)] == ["raised:True"] * 2
