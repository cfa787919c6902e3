"""ResNet-50 b256 training step fed from an LMDB through the native input path
(LMDBImageDataset -> LoaderConfig.make -> PinnedPrefetcher: native multi-threaded
LMDB gather into pinned ring buffers, side-stream H2D, device crop/flip/normalise)
vs the device-resident synthetic batch of bench.py.  Verdict r1 item 6."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from torchbooster_amd import models, utils
from torchbooster_amd.config import LoaderConfig
from torchbooster_amd.data import DeviceAugment, LMDBImageDataset, PinnedPrefetcher
from torchbooster_amd.ops.loss import cross_entropy_accuracy
from torchbooster_amd.ops.optim import FusedAdamW
from torchbooster_amd.scheduler import CycleScheduler

N_REC, B, STEPS, WARM = int(os.environ.get("N_REC", "2048")), 256, 20, 5
path = os.environ.get("LMDB_PATH", "/tmp/tbamd_imagenet_lmdb")
t0 = time.time()
if not os.path.exists(os.path.join(path, "data.mdb")):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, size=(N_REC, 224, 224, 3), dtype=np.uint8)
    LMDBImageDataset.prepare(path, imgs, rng.integers(0, 1000, size=N_REC))
    del imgs
print(f"[lmdb] {N_REC} records ready in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)

utils.boost(True)
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = models.resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-2)
sched = CycleScheduler(opt, 1e-3, 10_000, warmup=100, decay=("lin", "cos"))
ds = LMDBImageDataset(path, transform=DeviceAugment(hflip=True, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)))
loader = LoaderConfig(batch_size=B, drop_last=True, pin_memory=True).make(ds, shuffle=True)
assert isinstance(loader, PinnedPrefetcher), type(loader)
epoch = [0]
it = [iter(loader)]


def batch():
    try:
        return next(it[0])
    except StopIteration:
        epoch[0] += 1
        loader.set_epoch(epoch[0])
        it[0] = iter(loader)
        return next(it[0])


x0 = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y0 = torch.randint(0, 1000, (B,), device=dev)


def step(src):
    x, y = batch() if src == "lmdb" else (x0, y0)
    loss, _ = cross_entropy_accuracy(model(x), y, 0.1)
    utils.step(loss, opt, sched, clip=1.0)
    return loss


res = {}
for src in ("device", "lmdb", "device", "lmdb"):
    for _ in range(WARM):
        step(src)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(STEPS):
        step(src)
    torch.cuda.synchronize()
    res.setdefault(src, []).append(B * STEPS / (time.perf_counter() - t))
# the input path alone
torch.cuda.synchronize()
t = time.perf_counter()
n = 0
for _ in range(20):
    x, y = batch()
    n += x.shape[0]
torch.cuda.synchronize()
out = {"model": "resnet50", "batch": B, "records": N_REC, "img_s_device_resident": round(max(res["device"]), 1),
       "img_s_lmdb_pipeline": round(max(res["lmdb"]), 1), "loader_only_img_s": round(n / (time.perf_counter() - t), 1)}
out["lmdb_vs_device"] = round(out["img_s_lmdb_pipeline"] / out["img_s_device_resident"], 4)
print(json.dumps(out), flush=True)
