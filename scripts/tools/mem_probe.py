"""Device memory across training steps (leak probe): ResNet-50 b256 native step on a device-resident
batch, then on batches from the LMDB -> LoaderConfig -> PinnedPrefetcher path; prints
memory_allocated after every few steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from torchbooster_amd import models, utils  # noqa: E402
from torchbooster_amd.config import LoaderConfig  # noqa: E402
from torchbooster_amd.data import DeviceAugment, LMDBImageDataset  # noqa: E402
from torchbooster_amd.ops.loss import cross_entropy_accuracy  # noqa: E402
from torchbooster_amd.ops.optim import FusedAdamW  # noqa: E402

B = 256
utils.boost(True)
dev = torch.device("cuda", 0)
model = models.resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
x0 = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y0 = torch.randint(0, 1000, (B,), device=dev)
GB = 2 ** 30


def step(x, y):
    loss, _ = cross_entropy_accuracy(model(x), y, 0.1)
    utils.step(loss, opt, None, clip=1.0)


for i in range(int(os.environ.get("DEV_STEPS", "30"))):
    step(x0, y0)
    if i % 5 == 4:
        torch.cuda.synchronize()
        print(f"device step {i + 1}: allocated {torch.cuda.memory_allocated() / GB:.2f} GiB "
              f"reserved {torch.cuda.memory_reserved() / GB:.2f} GiB", flush=True)
path = "/tmp/tbamd_probe_lmdb"
if not os.path.exists(os.path.join(path, "data.mdb")):
    rng = np.random.default_rng(0)
    LMDBImageDataset.prepare(path, rng.integers(0, 256, size=(1024, 224, 224, 3), dtype=np.uint8),
                             rng.integers(0, 1000, size=1024))
ds = LMDBImageDataset(path, transform=DeviceAugment(hflip=True, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)))
loader = LoaderConfig(batch_size=B, drop_last=True, pin_memory=True).make(ds, shuffle=True)
it = iter(loader)
for i in range(int(os.environ.get("LMDB_STEPS", "20"))):
    try:
        x, y = next(it)
    except StopIteration:
        it = iter(loader)
        x, y = next(it)
    if i == 0:
        print("lmdb batch", x.shape, x.dtype, x.stride(), x.is_contiguous(memory_format=torch.channels_last), flush=True)
    step(x, y)
    if i % 5 == 4 or i < 3:
        torch.cuda.synchronize()
        print(f"lmdb step {i + 1}: allocated {torch.cuda.memory_allocated() / GB:.2f} GiB "
              f"reserved {torch.cuda.memory_reserved() / GB:.2f} GiB", flush=True)
