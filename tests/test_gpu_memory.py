"""Device memory must not grow across training steps (no reference cycles holding a step's
activations until a full gc pass): the bottleneck's lazy downsample placeholder once pointed back at
its LazyAct, which kept every step's graph context alive -- ~5 GB per ResNet-50 b256 step, an OOM
after ~55 steps on a 288 GB MI355X."""
import gc

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd import models, utils  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402


@pytest.mark.parametrize("name", ["resnet50", "stock_resnet50", "vit_tiny"])
def test_no_memory_growth_across_steps(name):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    if name == "stock_resnet50":
        from torchbooster_amd.models import tv
        from torchbooster_amd.nativize import nativize

        model = nativize(tv.resnet50(num_classes=100).to(dev).to(memory_format=torch.channels_last)
                         .to(torch.bfloat16))
    elif name == "vit_tiny":
        model = models.vit.vit_tiny(num_classes=100, image=32).to(dev).to(torch.bfloat16)
    else:
        model = getattr(models, name)(num_classes=100).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = FusedAdamW(model.parameters(), lr=1e-3)
    img = 32 if name == "vit_tiny" else 96
    x = torch.randn(16, 3, img, img, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (16,), device=dev)

    def step():
        loss, _ = cross_entropy_accuracy(model(x), y, 0.1)
        utils.step(loss, opt, None, clip=1.0)

    gc.collect()
    was = gc.isenabled()
    gc.disable()  # only reference counting frees memory: any cycle shows up as growth
    try:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        grown = torch.cuda.memory_allocated() - base
    finally:
        if was:
            gc.enable()
    assert grown <= 1 << 20, f"{grown / 2**20:.1f} MiB retained over 5 steps"
    gc.set_debug(gc.DEBUG_SAVEALL)
    try:
        gc.collect()
        cyc = [type(o).__name__ for o in gc.garbage if type(o).__name__ in
               ("LazyAct", "ResidualGradLink", "BnBwdLink", "GeluLink")]
    finally:
        gc.set_debug(0)
        gc.garbage.clear()
    assert not cyc, cyc
