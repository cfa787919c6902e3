"""One-shot all-reduce over IPC-mapped peer buffers (csrc/oneshot.hip, parallel/oneshot.py;
SURVEY.md §5.8 (c)): two processes share the one GPU of the box (IPC handles
map within a device too), exchange handles over a gloo group, and the one-shot result must be
bit-identical to ``tdist.all_reduce`` for fp32 and bf16 buffers of 4 KiB - 1 MiB; the native DDP
wrapper routed through it gives rank-identical gradients equal to the ring path's.
Reference: the GAN / VAE gradient buckets (examples/img_gen/gan/gan.py:31-49,102-113)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd import distributed as dist  # noqa: E402

SIZES = [4 << 10, 64 << 10, 256 << 10, 1 << 20]


def _worker(rank, world, port, q):
    try:
        os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        import torch.distributed as tdist

        torch.cuda.set_device(0)
        tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        from torchbooster_amd.parallel.oneshot import OneShotAllReduce

        ar = OneShotAllReduce(capacity_mb=1.0)
        res = []
        for dt in (torch.float32, torch.bfloat16):
            for nbytes in SIZES:
                n = nbytes // torch.tensor([], dtype=dt).element_size()
                g = torch.Generator(device="cuda").manual_seed(100 * rank + n)
                x = torch.randn(n, device="cuda", generator=g).to(dt)
                # reference: every rank's buffer, summed in f32 in rank order 0..world-1 (the
                # kernel's order), rounded once
                parts = [torch.empty_like(x).cpu() for _ in range(world)]
                tdist.all_gather(parts, x.cpu())
                acc = torch.zeros(n, dtype=torch.float32)
                for p_ in parts:
                    acc = acc + p_.float()
                ref = acc.to(dt).cuda()
                ref_mean = (acc * (1.0 / world)).to(dt).cuda()
                out = torch.empty_like(x)
                for _ in range(3):  # repeated calls: epochs / double buffering
                    ar.all_reduce(x, out=out)
                mean = ar.all_reduce(x.clone(), average=True)
                torch.cuda.synchronize()
                res.append((str(dt), nbytes, bool(torch.equal(out, ref)), bool(torch.equal(mean, ref_mean))))
        ar.check()
        # the native DDP wrapper with every bucket on the one-shot path vs the ring (gloo) path
        from torchbooster_amd.parallel import DistributedDataParallel

        def grads(oneshot_mb):
            torch.manual_seed(0)
            m = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.GELU(), torch.nn.Linear(512, 64)).cuda()
            ddp = DistributedDataParallel(m, bucket_cap_mb=0.25, first_bucket_mb=0.0625, oneshot_mb=oneshot_mb)
            torch.manual_seed(1 + rank)
            x = torch.randn(32, 256, device="cuda")
            ddp(x).square().mean().backward()
            torch.cuda.synchronize()
            return torch.cat([p.grad.reshape(-1) for p in m.parameters()]).cpu()

        g_os = grads(1.0)
        g_ring = grads(0.0)
        # a peer that never arrives fails LOUDLY -- the output chunk is NaN-poisoned and
        # check() raises (host-pinned error word, no sync); rank 1 skips the call
        late = OneShotAllReduce(capacity_mb=1.0, timeout_s=0.5)
        loud = True
        if rank == 0:
            y = torch.ones(4096, device="cuda")
            late.all_reduce(y)
            torch.cuda.synchronize()
            try:
                late.check()
                loud = False
            except RuntimeError:
                pass
            loud = loud and bool(torch.isnan(y).all())
        tdist.barrier()
        q.put((rank, res, g_os, g_ring, None if loud else "one-shot timeout was silent"))
        tdist.barrier()
        tdist.destroy_process_group()
    except BaseException as e:  # pragma: no cover - reported by the parent
        import traceback

        q.put((rank, None, None, None, traceback.format_exc()))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 4])
def test_oneshot_allreduce_matches_ring(world):
    """world 4 (four processes on the one GPU) exercises the [world][chunks] flag array and the
    epoch parity of the double-buffered staging beyond a pair."""
    port = dist.find_free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=200) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(60)
    for rank, res, g_os, g_ring, err in out:
        assert err is None, err
        bad = [r for r in res if not (r[2] and r[3])]
        assert not bad, bad
        # one-shot sums in rank order on every rank: rank-identical, and equal to the ring path
        assert torch.equal(g_os, out[0][2])
        assert torch.allclose(g_os, g_ring, rtol=1e-6, atol=1e-7), (g_os - g_ring).abs().max()
    for p in procs:
        assert p.exitcode == 0
