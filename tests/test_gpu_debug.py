"""Debug modes: the bounds-checked build (_C_bounds.so, TBAMD_BOUNDS=1)
flags a logically out-of-range device access and raises naming the op, runs the real
kernels without false positives, and TBAMD_LAUNCH_BLOCKING=1 synchronises after each op.
Each mode runs in a child process (the loader picks the library at import)."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code: str, **env) -> subprocess.CompletedProcess:
    e = dict(os.environ, **env)
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], cwd=ROOT, env=e, capture_output=True,
                          text=True, timeout=300)


def test_bounds_build_flags_and_names_the_op():
    r = _run("""
        import torch
        from torchbooster_amd.ops._ext import native
        C = native()
        assert C.bounds_enabled()
        x = torch.arange(1024, device="cuda", dtype=torch.float32)
        assert C.bounds_probe(x, 5).item() == 5.0
        try:
            C.bounds_probe(x[:16], 20)   # inside the allocation, outside the tensor
        except RuntimeError as e:
            assert "bounds_probe" in str(e) and "out-of-bounds" in str(e), e
            print("RAISED")
        """, TBAMD_BOUNDS="1")
    assert r.returncode == 0 and "RAISED" in r.stdout, r.stderr[-2000:]


def test_bounds_build_runs_real_kernels_clean():
    r = _run("""
        import torch, torch.nn.functional as F
        from torchbooster_amd.ops._ext import native
        from torchbooster_amd.ops.conv import Conv2d
        from torchbooster_amd.ops import gemm as G
        C = native()
        torch.manual_seed(0)
        conv = Conv2d(64, 128, 3, 1, 1, bias=False).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
        x = torch.randn(4, 64, 16, 16, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_()
        conv(x).float().square().mean().backward()
        small = Conv2d(3, 8, 9, 1, 4, padding_mode="reflect").cuda()
        xs = torch.randn(2, 3, 20, 20, device="cuda").requires_grad_()
        small(xs).square().mean().backward()
        a = torch.randn(300, 256, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(192, 256, device="cuda", dtype=torch.bfloat16)
        y = G.mm_nt(a, w)
        assert ((y.float() - a.float() @ w.float().t()).norm() / (a.float() @ w.float().t()).norm()) < 1e-2
        print("CLEAN")
        """, TBAMD_BOUNDS="1")
    assert r.returncode == 0 and "CLEAN" in r.stdout, r.stderr[-3000:]


def test_launch_blocking_mode():
    r = _run("""
        import torch
        from torchbooster_amd.ops._ext import native
        C = native()
        assert type(C).__name__ == "_Checked" and not C.bounds_enabled()
        x = torch.arange(64, device="cuda", dtype=torch.float32)
        assert C.bounds_probe(x, 3).item() == 3.0
        print("OK", C.__file__)
        """, TBAMD_LAUNCH_BLOCKING="1")
    assert r.returncode == 0 and "OK" in r.stdout and "_C." in r.stdout, r.stderr[-2000:]
