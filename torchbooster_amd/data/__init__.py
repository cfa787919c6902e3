"""Data sources and the device input pipeline.

* :class:`SyntheticImageDataset` / :class:`SyntheticSplitDataset` — deterministic
  synthetic stand-ins for MNIST / CIFAR-10 / ImageNet / COCO (there is no network
  here; ``DatasetConfig`` resolves the reference's dataset names to these when
  no local copy exists).
* :class:`LMDBImageDataset` — fixed-shape uint8 HWC images + int64 labels in an
  LMDB file (``prepare`` writes one), on the native reader.
* :class:`PinnedPrefetcher` — the MI355X input path: batches are
  gathered into pinned host ring buffers (natively, from LMDB, GIL released),
  copied H2D with ``non_blocking`` on a side HIP stream, and crop/flip/normalised
  to bf16 NHWC by a HIP kernel on the compute stream, ``depth`` batches ahead.
"""
from __future__ import annotations

import math
import os
import struct
import threading
from typing import Any, Callable, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from torchbooster_amd.dataset import BaseDataset, Split

__all__ = ["SyntheticImageDataset", "LMDBImageDataset", "PinnedPrefetcher", "device_normalize",
           "make_named_dataset", "KNOWN_SHAPES"]

# name -> (C, H, W, num_classes, train_len, test_len)
KNOWN_SHAPES = {
    "mnist": (1, 28, 28, 10, 60000, 10000),
    "cifar10": (3, 32, 32, 10, 50000, 10000),
    "cifar100": (3, 32, 32, 100, 50000, 10000),
    "imagenet": (3, 224, 224, 1000, 1281167, 50000),
    "coco": (3, 256, 256, 1, 118287, 5000),
}


class SyntheticImageDataset(Dataset):
    """Deterministic random images (uint8-valued, returned as float in [0, 1]
    CHW like ``ToTensor``) and labels; item ``i`` depends only on (seed, i)."""

    def __init__(self, length: int, shape=(3, 32, 32), num_classes: int = 10, seed: int = 0,
                 transform: Optional[Callable] = None, as_uint8: bool = False) -> None:
        self.length = int(length)
        self.shape = tuple(shape)
        self.num_classes = num_classes
        self.seed = seed
        self.transform = transform
        self.as_uint8 = as_uint8

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int):
        if i < 0 or i >= self.length:
            raise IndexError(i)
        g = np.random.default_rng(self.seed * 1_000_003 + i)
        img = g.integers(0, 256, size=self.shape, dtype=np.uint8)
        label = int(g.integers(0, self.num_classes))
        x = torch.from_numpy(img)
        if not self.as_uint8:
            x = x.float().div_(255.0)
        if self.transform is not None:
            x = self.transform(x)
        return x, label


class LMDBImageDataset(BaseDataset):
    """uint8 HWC images + int64 labels in LMDB: record ``str(i)`` =
    ``<q label><H*W*C bytes>``; ``b"shape"`` = ``"H,W,C"``."""

    HEADER = 8

    def __init__(self, path, transform: Optional[Callable] = None, **kw) -> None:
        super().__init__(path, transform, **kw)
        self._shape = None

    @property
    def shape(self) -> Tuple[int, int, int]:
        if self._shape is None:
            h, w, c = (int(v) for v in self.lmdb_reader.get(b"shape").decode().split(","))
            self._shape = (h, w, c)
        return self._shape

    @property
    def record_bytes(self) -> int:
        h, w, c = self.shape
        return self.HEADER + h * w * c

    def __getitem__(self, idx: int):
        raw = self.lmdb_reader[idx]
        label = struct.unpack_from("<q", raw, 0)[0]
        h, w, c = self.shape
        img = torch.frombuffer(bytearray(raw[self.HEADER:]), dtype=torch.uint8).view(h, w, c).permute(2, 0, 1)
        x = img.float().div_(255.0)
        if self.transform is not None:
            x = self.transform(x)
        return x, label

    @classmethod
    def prepare(cls, path, images, labels) -> int:
        """Write ``images`` (uint8 [N, H, W, C] array/tensor) and ``labels`` to ``path``."""
        from torchbooster_amd.lmdb import write_lmdb

        images = torch.as_tensor(np.asarray(images), dtype=torch.uint8)
        n, h, w, c = images.shape
        labels = [int(v) for v in labels]
        items = [(str(i), struct.pack("<q", labels[i]) + images[i].contiguous().numpy().tobytes())
                 for i in range(n)]
        items.append((b"shape", f"{h},{w},{c}".encode()))
        return write_lmdb(str(path), items, length=n)


def device_normalize(images_u8: torch.Tensor, mean: Sequence[float], std: Sequence[float],
                     out_hw: Optional[Tuple[int, int]] = None, offsets: Optional[torch.Tensor] = None,
                     flip: Optional[torch.Tensor] = None, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """uint8 [N, H, W, C] (device) -> normalised [N, C, Ho, Wo] channels_last.
    Optional per-image crop offsets [N, 2] (may be negative: reflect padding)
    and horizontal flips [N]."""
    N, H, W, C = images_u8.shape
    Ho, Wo = out_hw or (H, W)
    mean_t = torch.tensor(mean, dtype=torch.float32)
    istd = 1.0 / torch.tensor(std, dtype=torch.float32)
    if images_u8.is_cuda:
        from torchbooster_amd.ops._ext import native

        return native().u8_crop_flip_normalize(images_u8, Ho, Wo, offsets, flip, mean_t, istd, dtype)
    # CPU reference
    x = images_u8.permute(0, 3, 1, 2).float() / 255.0
    out = torch.empty(N, C, Ho, Wo)
    for n in range(N):
        oy, ox = (int(offsets[n, 0]), int(offsets[n, 1])) if offsets is not None else (0, 0)
        ys = torch.arange(Ho) + oy
        xs = torch.arange(Wo)
        if flip is not None and bool(flip[n]):
            xs = Wo - 1 - xs
        xs = xs + ox
        ys = torch.where(ys < 0, -ys, ys)
        ys = torch.where(ys >= H, 2 * H - 2 - ys, ys)
        xs = torch.where(xs < 0, -xs, xs)
        xs = torch.where(xs >= W, 2 * W - 2 - xs, xs)
        out[n] = x[n][:, ys][:, :, xs]
    out = (out - mean_t.view(1, C, 1, 1)) * istd.view(1, C, 1, 1)
    return out.to(dtype).contiguous(memory_format=torch.channels_last)


class PinnedPrefetcher:
    """Asynchronous host->device batch pipeline.

    ``fetch(indices, out_u8)`` fills a pinned uint8 ``[B, record_bytes]`` buffer
    (for :class:`LMDBImageDataset` this is the native multi-threaded LMDB
    ``gather``).  A background thread fills ``depth`` pinned slots; each slot is
    copied to the device on a dedicated HIP stream (``non_blocking``) and the
    compute stream waits on that copy's event only when the batch is consumed.
    Yields ``(images [B, C, Ho, Wo] bf16 channels_last, labels int64)``.
    """

    def __init__(self, dataset: LMDBImageDataset, batch_size: int, device=None, depth: int = 3,
                 shuffle: bool = True, drop_last: bool = True, seed: int = 0, mean=(0.485, 0.456, 0.406),
                 std=(0.229, 0.224, 0.225), crop: Optional[Tuple[int, int]] = None, pad: int = 0,
                 random_flip: bool = False, dtype=torch.bfloat16, threads: int = 8, rank: int = 0,
                 world_size: int = 1) -> None:
        self.ds = dataset
        self.B = batch_size
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.depth = depth
        self.shuffle, self.drop_last, self.seed = shuffle, drop_last, seed
        self.mean, self.std = mean, std
        self.crop, self.pad, self.random_flip = crop, pad, random_flip
        self.dtype = dtype
        self.threads = threads
        self.rank, self.world = rank, world_size
        self.epoch = 0
        h, w, c = dataset.shape
        self.hwc = (h, w, c)
        self.rec = dataset.record_bytes
        pin = self.device.type == "cuda"
        self.host = [torch.empty(self.B, self.rec, dtype=torch.uint8, pin_memory=pin) for _ in range(depth)]
        self.stream = torch.cuda.Stream(self.device) if pin else None

    def set_epoch(self, e: int) -> None:
        self.epoch = e

    def _order(self) -> List[int]:
        n = len(self.ds)
        g = np.random.default_rng(self.seed + self.epoch)
        idx = g.permutation(n) if self.shuffle else np.arange(n)
        per = n // self.world if self.drop_last else math.ceil(n / self.world)
        idx = idx[self.rank * per:(self.rank + 1) * per]
        nb = len(idx) // self.B if self.drop_last else math.ceil(len(idx) / self.B)
        return [idx[i * self.B:(i + 1) * self.B].tolist() for i in range(nb)]

    def __len__(self) -> int:
        return len(self._order())

    def _fill(self, slot: int, batch: List[int]) -> None:
        buf = self.host[slot][: len(batch)]
        self.ds.lmdb_reader.gather(batch, buf, self.threads)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        batches = self._order()
        g = np.random.default_rng(self.seed * 7919 + self.epoch)
        h, w, c = self.hwc
        Ho, Wo = self.crop or (h, w)
        filled = [threading.Event() for _ in range(self.depth)]
        free = [threading.Event() for _ in range(self.depth)]
        for e in free:
            e.set()
        stop = [False]

        def producer():
            for bi, b in enumerate(batches):
                s = bi % self.depth
                free[s].wait()
                if stop[0]:
                    return
                free[s].clear()
                self._fill(s, b)
                filled[s].set()

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        pending = []
        try:
            for bi, b in enumerate(batches):
                s = bi % self.depth
                filled[s].wait()
                filled[s].clear()
                n = len(b)
                host = self.host[s][:n]
                if self.stream is not None:
                    with torch.cuda.stream(self.stream):
                        dev = host.to(self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                    torch.cuda.current_stream(self.device).wait_event(ev)
                    dev.record_stream(torch.cuda.current_stream(self.device))
                    # host slot is reusable once the copy is done
                    pending.append((ev, s))
                    while pending and pending[0][0].query():
                        free[pending.pop(0)[1]].set()
                    if len(pending) >= self.depth - 1:
                        e0, s0 = pending.pop(0)
                        e0.synchronize()
                        free[s0].set()
                else:
                    dev = host.clone()
                    free[s].set()
                labels = dev[:, :8].contiguous().view(torch.int64).view(n)
                imgs = dev[:, 8:].view(n, h, w, c)
                offs = flip = None
                if self.crop is not None or self.pad:
                    oy = g.integers(-self.pad, h - Ho + self.pad + 1, size=n)
                    ox = g.integers(-self.pad, w - Wo + self.pad + 1, size=n)
                    offs = torch.from_numpy(np.stack([oy, ox], 1).astype(np.int32))
                if self.random_flip:
                    flip = torch.from_numpy(g.integers(0, 2, size=n).astype(np.uint8))
                x = device_normalize(imgs, self.mean, self.std, (Ho, Wo), offs, flip, self.dtype)
                yield x, labels
        finally:
            stop[0] = True
            for e in free:
                e.set()
            th.join(timeout=5)
            for ev, s in pending:
                ev.synchronize()


def make_named_dataset(name: str, root: str, split: Split, **kwargs) -> Optional[Dataset]:
    """Resolve a reference dataset name without network access.

    1. ``root`` holding an LMDB (``data.mdb``) -> :class:`LMDBImageDataset`;
    2. ``synthetic:<name>`` or a known name (mnist/cifar10/cifar100/imagenet/coco)
       when ``TBAMD_SYNTHETIC_DATA`` is not ``0`` -> :class:`SyntheticImageDataset`
       of that dataset's shape and size;
    3. otherwise None (torchvision / torchtext / HF are tried next).
    """
    if root and os.path.exists(os.path.join(root, "data.mdb")):
        return LMDBImageDataset(root, transform=kwargs.get("transform"))
    key = name.lower()
    synthetic = key.startswith("synthetic:")
    if synthetic:
        key = key.split(":", 1)[1]
    if key in KNOWN_SHAPES and (synthetic or os.environ.get("TBAMD_SYNTHETIC_DATA", "1") != "0"):
        c, h, w, k, ntr, nte = KNOWN_SHAPES[key]
        n = ntr if split == Split.TRAIN else nte
        n = int(os.environ.get("TBAMD_SYNTHETIC_LEN", n))
        seed = {Split.TRAIN: 0, Split.VALID: 1, Split.TEST: 2}[split]
        return SyntheticImageDataset(n, (c, h, w), k, seed=seed, transform=kwargs.get("transform"))
    return None
