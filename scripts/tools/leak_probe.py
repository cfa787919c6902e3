"""Is the per-step device-memory growth cyclic garbage?  ResNet-50 b256 native steps: 6 plain, 6 with
gc.collect() after each, then one step under gc.DEBUG_SAVEALL: the types in the collected cycles and
the tensors they held."""
import collections
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from torchbooster_amd import models, utils  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

B = int(os.environ.get("B", "256"))
MODEL = os.environ.get("MODEL", "resnet50")
utils.boost(True)
dev = torch.device("cuda", 0)
if MODEL == "stock_resnet50":
    from torchbooster_amd.models import tv
    from torchbooster_amd.nativize import nativize
    model = nativize(tv.resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16))
else:
    model = getattr(models, MODEL)(num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
x0 = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y0 = torch.randint(0, 1000, (B,), device=dev)
GB = 2 ** 30


def step():
    loss, _ = cross_entropy_accuracy(model(x0), y0, 0.1)
    utils.step(loss, opt, None, clip=1.0)


def mem(tag):
    torch.cuda.synchronize()
    print(f"{tag}: allocated {torch.cuda.memory_allocated() / GB:.2f} GiB", flush=True)


for i in range(6):
    step()
    mem(f"plain step {i + 1}")
for i in range(6):
    step()
    n = gc.collect()
    mem(f"gc step {i + 1} (collected {n})")
gc.collect()
gc.set_debug(gc.DEBUG_SAVEALL)
step()
gc.collect()
types = collections.Counter(type(o).__name__ for o in gc.garbage)
print("cyclic garbage of one step:", types.most_common(25), flush=True)
tens = [o for o in gc.garbage if isinstance(o, torch.Tensor)]
print(f"tensors in cycles: {len(tens)}, {sum(t.untyped_storage().nbytes() for t in tens if t.is_cuda) / GB:.2f} GiB "
      "of storage", flush=True)
owners = collections.Counter()
for o in gc.garbage:
    if type(o).__name__ in ("LazyAct", "ResidualGradLink", "BnBwdLink", "GeluLink"):
        owners[type(o).__name__] += 1
    if isinstance(o, dict) and ("_tb_lazy_affine" in o):
        owners["tensor.__dict__ with _tb_lazy_affine"] += 1
print("framework objects in cycles:", dict(owners), flush=True)
for o in gc.garbage[:0]:
    pass
gc.set_debug(0)
gc.garbage.clear()
