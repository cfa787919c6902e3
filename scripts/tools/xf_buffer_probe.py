"""Running-statistics deviation of the lazy-BN (XF) ResNet-50 step vs the materialised step, each
measured against the fp32 ATen step from the same init (the setting of
tests/test_gpu_xf.py::test_resnet50_lazy_bn_matches_materialised).  Prints, per BN buffer, the max
abs deviation of each bf16 path from fp32 and of the two bf16 paths from each other, plus a rerun
of each bf16 path (determinism)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from torchbooster_amd import models  # noqa: E402
from torchbooster_amd.models import resnet as RN  # noqa: E402


def main():
    torch.manual_seed(0)
    m0 = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).train()
    state = {k: v.clone() for k, v in m0.state_dict().items()}
    x = torch.randn(48, 3, 160, 160, device="cuda").contiguous(memory_format=torch.channels_last)
    t = torch.randint(0, 10, (48,), device="cuda")
    RN._LAZY_DS = False

    def run(lazy, dtype=torch.bfloat16):
        RN._LAZY_BN = lazy
        m = models.resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last).train()
        m.load_state_dict(state)
        m = m.to(dtype)
        loss = F.cross_entropy(m(x.to(dtype)).float(), t)
        loss.backward()
        torch.cuda.synchronize()
        bufs = [(n, b.detach().float().clone()) for n, b in m.named_buffers() if "running" in n]
        return loss.item(), bufs

    os.environ["TBAMD_FORCE_REFERENCE"] = "1"
    lr, br = run(False, torch.float32)
    del os.environ["TBAMD_FORCE_REFERENCE"]
    l0, b0 = run(False)
    l0b, b0b = run(False)
    l1, b1 = run(True)
    l1b, b1b = run(True)
    print(f"loss fp32 {lr:.5f} materialised {l0:.5f}/{l0b:.5f} lazy {l1:.5f}/{l1b:.5f}")
    worst = []
    for (n, r), (_, a), (_, a2), (_, b), (_, b2) in zip(br, b0, b0b, b1, b1b):
        e0 = (a - r).abs().max().item()
        e1 = (b - r).abs().max().item()
        d = (a - b).abs()
        tol = 1e-3 + 2e-2 * b.abs()
        bad = int((d > tol).sum().item())
        worst.append((bad, n, e0, e1, d.max().item(), (a - a2).abs().max().item(), (b - b2).abs().max().item()))
    print("buffer  n_outside_test_tol  |mat-fp32|  |lazy-fp32|  |mat-lazy|  |mat rerun|  |lazy rerun|")
    for w in worst:
        if w[0] or w[2] > 2e-3 or w[3] > 2e-3:
            print(f"{w[1]:40s} {w[0]:4d}  {w[2]:.5f}  {w[3]:.5f}  {w[4]:.5f}  {w[5]:.5f}  {w[6]:.5f}")
    tot0 = sum(w[2] for w in worst)
    tot1 = sum(w[3] for w in worst)
    print(f"sum over buffers of max |dev from fp32|: materialised {tot0:.4f} lazy {tot1:.4f}")


if __name__ == "__main__":
    main()
