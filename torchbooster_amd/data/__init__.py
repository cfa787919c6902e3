"""Data sources and the device input pipeline.

* :class:`SyntheticImageDataset` / :class:`SyntheticSplitDataset` — deterministic
  synthetic stand-ins for MNIST / CIFAR-10 / ImageNet / COCO (there is no network
  here; ``DatasetConfig`` resolves the reference's dataset names to these when
  no local copy exists).
* :class:`LMDBImageDataset` — fixed-shape uint8 HWC images + int64 labels in an
  LMDB file (``prepare`` writes one; :func:`pack_folder` streams an image folder
  into one), on the native reader.
* :class:`MNISTDataset` / :class:`CIFARBinaryDataset` / :class:`ImageFolderDataset`
  — the reference's own sources (MNIST idx files, CIFAR binary batches, COCO /
  painting image folders) without torchvision (data/readers.py).
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

__all__ = ["SyntheticImageDataset", "LMDBImageDataset", "PinnedPrefetcher", "shard_indices", "device_normalize",
           "make_named_dataset", "KNOWN_SHAPES", "DeviceAugment", "DeviceImageLoader", "device_loader",
           "MNISTDataset", "CIFARBinaryDataset", "ImageFolderDataset", "pack_folder"]

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

    def _item(self, i: int):
        g = np.random.default_rng(self.seed * 1_000_003 + i)
        img = g.integers(0, 256, size=self.shape, dtype=np.uint8)
        return img, int(g.integers(0, self.num_classes))

    def arrays_u8(self):
        """(uint8 [N, H, W, C], int64 [N]) of the whole dataset (the device loader's storage)."""
        imgs = np.empty((self.length,) + (self.shape[1], self.shape[2], self.shape[0]), dtype=np.uint8)
        labels = np.empty(self.length, dtype=np.int64)
        for i in range(self.length):
            im, lab = self._item(i)
            imgs[i] = im.transpose(1, 2, 0)
            labels[i] = lab
        return imgs, labels

    def __getitem__(self, i: int):
        if i < 0 or i >= self.length:
            raise IndexError(i)
        img, label = self._item(i)
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


def shard_indices(idx: np.ndarray, rank: int, world: int, drop_last: bool) -> np.ndarray:
    """``DistributedSampler``'s partition of an (already shuffled) index list: every
    rank gets the same count -- ``drop_last`` trims the tail to a multiple of
    ``world``, otherwise the list is padded by wrapping around -- and rank ``r``
    takes ``idx[r::world]``.  Equal per-rank batch counts keep DDP collectives in
    step (a short last rank would hang its peers)."""
    n = len(idx)
    if world <= 1:
        return idx
    if drop_last:
        idx = idx[: (n // world) * world]
    else:
        total = math.ceil(n / world) * world
        if total > n:
            reps = math.ceil(total / max(n, 1))
            idx = np.concatenate([idx] * reps)[:total] if n else idx
    return idx[rank::world]


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
                 world_size: int = 1, augment: Optional["DeviceAugment"] = None) -> None:
        self.augment = augment
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
        idx = shard_indices(g.permutation(n) if self.shuffle else np.arange(n), self.rank, self.world,
                            self.drop_last)
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
                if self.augment is not None and h * w * c <= 32768:
                    yield self.augment.apply(imgs, self.augment.params(n, h, w, g)), labels
                    continue
                if self.augment is not None:  # large images: crop / flip / normalise (no LDS pipeline)
                    a = self.augment
                    Ho, Wo = a.size or (h, w)
                    pad = a.padding
                    oy = g.integers(-pad, h - Ho + pad + 1, size=n)
                    ox = g.integers(-pad, w - Wo + pad + 1, size=n)
                    offs = torch.from_numpy(np.stack([oy, ox], 1).astype(np.int32))
                    flip = torch.from_numpy(g.integers(0, 2, size=n).astype(np.uint8)) if a.hflip else None
                    yield device_normalize(imgs, a.mean * (c // len(a.mean)), a.std * (c // len(a.std)), (Ho, Wo),
                                           offs, flip, a.dtype), labels
                    continue
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


def synthetic_for(name: str, split: Split, **kwargs) -> Optional[Dataset]:
    """:class:`SyntheticImageDataset` of a known dataset's shape and size (mnist /
    cifar10 / cifar100 / imagenet / coco), or None for an unknown name."""
    key = name.lower()
    if key.startswith("synthetic:"):
        key = key.split(":", 1)[1]
    if key.split(":", 1)[0] in _FOLDER_NAMES:  # an image folder that is not there: COCO-shaped stand-in
        key = "coco"
    if key not in KNOWN_SHAPES:
        return None
    c, h, w, k, ntr, nte = KNOWN_SHAPES[key]
    n = ntr if split == Split.TRAIN else nte
    n = int(os.environ.get("TBAMD_SYNTHETIC_LEN", n))
    seed = {Split.TRAIN: 0, Split.VALID: 1, Split.TEST: 2}[split]
    return SyntheticImageDataset(n, (c, h, w), k, seed=seed, transform=kwargs.get("transform"))


# image-folder dataset names: the generic ones, and the reference's COCO / paintings folders
# (online.yml / adain.yml name them "coco" / "paintings" with an ImageFolder root)
_FOLDER_NAMES = ("folder", "imagefolder", "image_folder", "coco", "paintings")


def _folder_path(name: str, root: str) -> Optional[str]:
    """The image folder a ``folder`` / ``folder:<path>`` dataset name points at: the explicit path,
    else ``root/<split>``, else ``root`` itself (the reference's ``ImageFolder(root=conf.root)``)."""
    low = name.lower()
    if ":" in name and low.split(":", 1)[0] in _FOLDER_NAMES:
        p = name.split(":", 1)[1]
        return p if os.path.isdir(p) else None
    for p in (root, os.path.dirname(root.rstrip("/")) if root else None):
        if p and os.path.isdir(p):
            return p
    return None


def make_named_dataset(name: str, root: str, split: Split, **kwargs) -> Optional[Dataset]:
    """Datasets this package resolves BEFORE the reference's sources (``root`` is
    ``<DatasetConfig.root>/<split>``, as in the reference, config.py:567):

    1. ``root`` holding an LMDB (``data.mdb``) -> :class:`LMDBImageDataset`;
    2. an explicit ``synthetic:<name>`` -> :class:`SyntheticImageDataset` of that
       dataset's shape and size;
    3. ``mnist`` (and the idx-format ``fashionmnist`` / ``kmnist``) / ``cifar10`` / ``cifar100``
       with their files under ``root`` (torchvision's layout, or flat), else under the dataset root
       -> the native readers of data/readers.py (idx files; CIFAR *binary* batches);
    4. ``folder`` / ``imagefolder`` / ``folder:<path>`` -> :class:`ImageFolderDataset`
       (``size`` kwarg: crop side, default 256);
    5. otherwise None (torchvision / torchtext / HF are tried next; a known name
       falls back to synthetic data only when ``TBAMD_SYNTHETIC_DATA=1`` asks for
       it, with a warning — ``DatasetConfig.make``).
    """
    from torchbooster_amd.data import readers as R

    if root and os.path.exists(os.path.join(root, "data.mdb")):
        return LMDBImageDataset(root, transform=kwargs.get("transform"))
    low = name.lower()
    if low.startswith("synthetic:"):
        return synthetic_for(name, split, **kwargs)
    tf = kwargs.get("transform")
    train = split is Split.TRAIN
    parent = os.path.dirname(root.rstrip("/")) if root else ""
    if low in ("mnist", "fashionmnist", "kmnist"):
        for r in (root, parent):
            if r and R.find_mnist(r, train) is not None:
                return R.MNISTDataset(r, train, transform=tf)
        return None
    if low in ("cifar10", "cifar100"):
        for r in (root, parent):
            if r and R.find_cifar(r, low, train) is not None:
                return R.CIFARBinaryDataset(r, low, train, transform=tf)
        return None
    if low.split(":", 1)[0] in _FOLDER_NAMES:
        path = _folder_path(name, root)
        if path is None:
            # a missing folder is a missing dataset: DatasetConfig.make falls through to its
            # logging.fatal + exit(1) (reference config.py:616-617), unless TBAMD_SYNTHETIC_DATA=1
            # asks for a COCO-shaped synthetic stand-in (synthetic_for maps folder names to "coco")
            return None
        return R.ImageFolderDataset(path, size=kwargs.get("size", 256), transform=tf,
                                    random_crop=bool(kwargs.get("random_crop", False)))
    return None


# ---------------------------------------------------------------------------------
# GPU training transforms + the device-resident loader

_RA_SIGNED = {1, 2, 3, 4, 5, 6, 7, 8, 9}


class DeviceAugment:
    """The reference's CIFAR training transform, run on the GPU.

    ``RandomCrop(size, padding, padding_mode="reflect")`` -> ``RandomHorizontalFlip``
    -> ``RandomRotation(rotate)`` -> ``RandAugment(num_ops, magnitude)`` ->
    ``ToTensor`` -> ``Normalize(mean, std)``
    (/root/reference/examples/img_cls/resnet/resnet.py:96-103), for uint8 HWC
    images: csrc/data.hip ``augment_u8_k`` does every stage for a whole batch in
    one launch (one workgroup per image, the image held in LDS), on random
    parameters drawn here on the host.  Used as a dataset ``transform`` it makes
    ``LoaderConfig.make`` build the device loader; called on one CHW float image
    (a CPU DataLoader) it runs :meth:`reference`, the same pipeline in NumPy."""

    def __init__(self, size: Optional[Tuple[int, int]] = None, padding: int = 0, hflip: bool = False,
                 rotate: float = 0.0, randaugment: bool = False, num_ops: int = 2, magnitude: int = 9,
                 mean: Sequence[float] = (0.5,), std: Sequence[float] = (0.5,), dtype=torch.bfloat16) -> None:
        self.size = None if size is None else ((size, size) if isinstance(size, int) else tuple(size))
        self.padding, self.hflip, self.rotate = int(padding), bool(hflip), float(rotate)
        self.randaugment, self.num_ops, self.magnitude = bool(randaugment), int(num_ops), int(magnitude)
        if self.randaugment and self.num_ops > 2:
            raise ValueError("DeviceAugment: at most 2 RandAugment ops")
        self.mean, self.std = tuple(float(v) for v in mean), tuple(float(v) for v in std)
        self.dtype = dtype

    def _ra_mag(self, op: int, H: int, W: int) -> float:
        b = self.magnitude / 30.0  # torchvision: 31 bins, value = linspace(lo, hi, 31)[magnitude]
        return {1: 0.3 * b, 2: 0.3 * b, 3: 150.0 / 331.0 * W * b, 4: 150.0 / 331.0 * H * b, 5: 30.0 * b,
                6: 0.9 * b, 7: 0.9 * b, 8: 0.9 * b, 9: 0.9 * b,
                10: float(8 - int(round(self.magnitude / 7.5))), 11: 255.0 - 255.0 * b}.get(op, 0.0)

    def params(self, B: int, H: int, W: int, rng: np.random.Generator) -> np.ndarray:
        """[B, 8] f32: oy, ox, flip, rotate_deg, op1, mag1, op2, mag2."""
        Ho, Wo = self.size or (H, W)
        p = np.zeros((B, 8), dtype=np.float32)
        if self.size is not None or self.padding:
            p[:, 0] = rng.integers(-self.padding, H - Ho + self.padding + 1, size=B)
            p[:, 1] = rng.integers(-self.padding, W - Wo + self.padding + 1, size=B)
        if self.hflip:
            p[:, 2] = rng.integers(0, 2, size=B)
        if self.rotate:
            p[:, 3] = rng.uniform(-self.rotate, self.rotate, size=B)
        if self.randaugment:
            for k in range(self.num_ops):
                ops = rng.integers(0, 14, size=B)
                sign = np.where(rng.integers(0, 2, size=B) == 1, -1.0, 1.0)
                mags = np.array([self._ra_mag(int(o), Ho, Wo) * (sign[i] if int(o) in _RA_SIGNED else 1.0)
                                 for i, o in enumerate(ops)], dtype=np.float32)
                p[:, 4 + 2 * k] = ops
                p[:, 5 + 2 * k] = mags
        return p

    def apply(self, images_u8: torch.Tensor, params: np.ndarray, src: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 [N, H, W, C] on the GPU (+ rows ``src``) -> normalised [B, C, Ho, Wo] channels_last."""
        from torchbooster_amd.ops._ext import native

        H, W, C = images_u8.shape[1:]
        Ho, Wo = self.size or (H, W)
        # the normalisation constants live on the device once: a per-batch copy from pageable host
        # memory would block the host until the GPU drained the previous step
        key = (images_u8.device, C)
        norm = getattr(self, "_norm", {}).get(key)
        if norm is None:
            mean = torch.tensor(self.mean * (C // len(self.mean)), dtype=torch.float32)
            istd = 1.0 / torch.tensor(self.std * (C // len(self.std)), dtype=torch.float32)
            norm = (mean.to(images_u8.device), istd.to(images_u8.device))
            self._norm = {**getattr(self, "_norm", {}), key: norm}
        mean, istd = norm
        pr = torch.from_numpy(params).pin_memory().to(images_u8.device, non_blocking=True)
        # geometry-only pipelines stream global -> global (any image size, one thread per pixel);
        # rotation / RandAugment run the LDS pipeline on the whole image
        crop_only = not self.rotate and not self.randaugment
        return native().augment_u8(images_u8, src, Ho, Wo, pr, mean, istd, self.dtype, crop_only)

    # ---------------------------------------------------------------- CPU reference
    @staticmethod
    def _warp(img: np.ndarray, m) -> np.ndarray:
        H, W, C = img.shape
        ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
        sx = np.rint(m[0] * xs + m[1] * ys + m[2]).astype(np.int64)
        sy = np.rint(m[3] * xs + m[4] * ys + m[5]).astype(np.int64)
        ok = (sx >= 0) & (sx < W) & (sy >= 0) & (sy < H)
        out = np.zeros_like(img)
        out[ok] = img[sy[ok], sx[ok]]
        return out

    @staticmethod
    def _rot(deg: float, H: int, W: int):
        a = np.float32(deg) * np.float32(0.017453292519943295)
        cs, sn = np.cos(a, dtype=np.float32), np.sin(a, dtype=np.float32)
        cx, cy = np.float32((W - 1) * 0.5), np.float32((H - 1) * 0.5)
        return [cs, -sn, cx - cs * cx + sn * cy, sn, cs, cy - sn * cx - cs * cy]

    @staticmethod
    def _gray(img: np.ndarray) -> np.ndarray:
        f = img.astype(np.float32)
        if img.shape[2] >= 3:
            return np.floor(np.float32(0.2989) * f[..., 0] + np.float32(0.587) * f[..., 1]
                            + np.float32(0.114) * f[..., 2])
        return f[..., 0]

    @classmethod
    def _op(cls, op: int, mag: float, img: np.ndarray) -> np.ndarray:
        H, W, C = img.shape
        f = img.astype(np.float32)
        mag = np.float32(mag)
        u8 = lambda v: np.clip(v, 0, 255).astype(np.uint8)  # noqa: E731 (truncation like the kernel)
        if op == 0:
            return img
        if op in (1, 2, 3, 4, 5):
            m = [1, 0, 0, 0, 1, 0]
            if op == 1:
                m[1] = -mag
            elif op == 2:
                m[3] = -mag
            elif op == 3:
                m[2] = -np.trunc(mag)
            elif op == 4:
                m[5] = -np.trunc(mag)
            else:
                m = cls._rot(mag, H, W)
            return cls._warp(img, m)
        if op == 6:
            return u8(f * (1 + mag))
        if op == 7:
            return u8((1 + mag) * f - mag * cls._gray(img)[..., None]) if C >= 3 else img
        if op == 8:
            mean = np.float32(cls._gray(img).sum(dtype=np.float32) / (H * W))
            return u8((1 + mag) * f - mag * mean)
        if op == 9:
            sm = f.copy()
            t = 4 * f[1:-1, 1:-1]
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    t = t + f[1 + dy:H - 1 + dy, 1 + dx:W - 1 + dx]
            sm[1:-1, 1:-1] = np.rint(t / np.float32(13))
            return u8((1 + mag) * f - mag * sm)
        if op == 10:
            return img & np.uint8(~((1 << (8 - int(mag))) - 1) & 0xFF)
        if op == 11:
            return np.where(f >= mag, 255 - img, img).astype(np.uint8)
        out = np.empty_like(img)
        for c in range(C):
            ch = img[..., c]
            if op == 12:
                lo, hi = float(ch.min()), float(ch.max())
                sc = np.float32(255.0 / (hi - lo)) if hi > lo else np.float32(1)
                off = np.float32(lo if hi > lo else 0)
                out[..., c] = u8((ch.astype(np.float32) - off) * sc)
            else:
                hist = np.bincount(ch.ravel(), minlength=256)
                nz = np.nonzero(hist)[0]
                step = (H * W - hist[nz[-1]]) // 255
                if step == 0:
                    out[..., c] = ch
                else:
                    lut = np.minimum(255, (np.concatenate([[0], np.cumsum(hist)[:-1]]) + step // 2) // step)
                    out[..., c] = lut[ch].astype(np.uint8)
        return out

    def reference(self, img_hwc: np.ndarray, p: np.ndarray) -> np.ndarray:
        """One uint8 HWC image through the pipeline with parameters ``p`` (f32 [8]) -> f32 CHW."""
        H, W, C = img_hwc.shape
        Ho, Wo = self.size or (H, W)
        ys = np.arange(Ho)[:, None] + int(p[0])
        xs = np.arange(Wo)[None, :]
        if p[2]:
            xs = Wo - 1 - xs
        xs = xs + int(p[1])
        ys = np.where(ys < 0, -ys, ys)
        ys = np.where(ys >= H, 2 * H - 2 - ys, ys)
        xs = np.where(xs < 0, -xs, xs)
        xs = np.where(xs >= W, 2 * W - 2 - xs, xs)
        img = img_hwc[ys, xs]
        if p[3]:
            img = self._warp(img, self._rot(float(p[3]), Ho, Wo))
        for k in range(2):
            img = self._op(int(p[4 + 2 * k]), float(p[5 + 2 * k]), img)
        mean = np.array(self.mean * (C // len(self.mean)), dtype=np.float32)
        std = np.array(self.std * (C // len(self.std)), dtype=np.float32)
        return ((img.astype(np.float32) / 255.0 - mean) / std).transpose(2, 0, 1)

    def __call__(self, x: torch.Tensor, rng: Optional[np.random.Generator] = None) -> torch.Tensor:
        """CPU path for a DataLoader: one CHW float image in [0, 1] (ToTensor layout)."""
        u8 = (x.detach().cpu().float() * 255.0).round().clamp(0, 255).to(torch.uint8).permute(1, 2, 0).numpy()
        rng = rng or np.random.default_rng(int(torch.randint(0, 2 ** 31 - 1, (1,))))
        p = self.params(1, u8.shape[0], u8.shape[1], rng)[0]
        return torch.from_numpy(self.reference(u8, p))


class DeviceImageLoader:
    """A whole uint8 image dataset resident in HBM (CIFAR-10 is 150 MB of a 288 GB
    device) served as augmented batches with no host work per sample: each step
    draws a permutation slice + per-image augmentation parameters on the host
    (``B x 8`` floats) and ONE kernel gathers, augments and normalises the batch
    (:class:`DeviceAugment`).  Yields ``(images [B, C, Ho, Wo], labels [B])`` on
    the device; ``set_epoch`` reshuffles (distributed: :func:`shard_indices`,
    ``DistributedSampler``'s rank-strided, equal-length shards)."""

    def __init__(self, images_u8: torch.Tensor, labels: torch.Tensor, batch_size: int,
                 augment: Optional["DeviceAugment"] = None, shuffle: bool = True, drop_last: bool = True,
                 seed: int = 0, rank: int = 0, world_size: int = 1, length: Optional[int] = None) -> None:
        # length > len(images): a pooled dataset (a synthetic ImageNet-shape set keeps a pool of
        # distinct images resident; sample i is image / label i % pool)
        self.images, self.labels = images_u8, labels
        self.length = int(length) if length is not None else len(labels)
        self.B = int(batch_size)
        self.augment = augment or DeviceAugment()
        self.shuffle, self.drop_last, self.seed = shuffle, drop_last, seed
        self.rank, self.world = rank, world_size
        self.epoch = 0

    @property
    def sampler(self):
        return self

    def set_epoch(self, e: int) -> None:
        self.epoch = int(e)

    def _order(self) -> np.ndarray:
        n = self.length
        idx = np.random.default_rng(self.seed + self.epoch).permutation(n) if self.shuffle else np.arange(n)
        return shard_indices(idx, self.rank, self.world, self.drop_last)

    def __len__(self) -> int:
        m = len(self._order())
        return m // self.B if self.drop_last else math.ceil(m / self.B)

    def __iter__(self):
        idx = self._order()
        g = np.random.default_rng((self.seed + 1) * 7919 + self.epoch)
        H, W = self.images.shape[1], self.images.shape[2]
        dev = self.images.device
        for b in range(len(self)):
            rows = idx[b * self.B:(b + 1) * self.B]
            if self.length != len(self.labels):
                rows = rows % len(self.labels)
            src = torch.from_numpy(rows.astype(np.int32)).pin_memory().to(dev, non_blocking=True)
            x = self.augment.apply(self.images, self.augment.params(len(rows), H, W, g), src)
            yield x, self.labels.index_select(0, src.long())


_SYNTH_POOL_BYTES = int(os.environ.get("TBAMD_SYNTH_POOL_MB", "512")) << 20


def device_loader(dataset, batch_size: int, shuffle: bool, drop_last: bool, device=None, rank: int = 0,
                  world_size: int = 1, seed: int = 0):
    """The native loader for ``dataset`` when its transform is a :class:`DeviceAugment`
    (None otherwise): LMDB image datasets stream through :class:`PinnedPrefetcher`;
    in-memory image datasets (``arrays_u8()``, or torchvision-style ``data`` /
    ``targets``) are moved to the device once and served by :class:`DeviceImageLoader`."""
    aug = getattr(dataset, "transform", None)
    if not isinstance(aug, DeviceAugment) or not torch.cuda.is_available():
        return None
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if isinstance(dataset, LMDBImageDataset):
        return PinnedPrefetcher(dataset, batch_size, device, shuffle=shuffle, drop_last=drop_last, seed=seed,
                                rank=rank, world_size=world_size, augment=aug)
    length = None
    if isinstance(dataset, SyntheticImageDataset) and len(dataset) * int(np.prod(dataset.shape)) > _SYNTH_POOL_BYTES:
        # synthetic ImageNet-shape sets (1.28 M x 150 KB): a resident pool of distinct images
        pool = max(1, min(len(dataset), _SYNTH_POOL_BYTES // int(np.prod(dataset.shape))))
        imgs, labels = SyntheticImageDataset(pool, dataset.shape, dataset.num_classes, dataset.seed).arrays_u8()
        length = len(dataset)
    elif hasattr(dataset, "arrays_u8"):
        imgs, labels = dataset.arrays_u8()
    elif hasattr(dataset, "data") and hasattr(dataset, "targets"):
        imgs, labels = np.asarray(dataset.data), np.asarray(dataset.targets)
        if imgs.ndim == 3:
            imgs = imgs[..., None]
    else:
        return None
    images = torch.from_numpy(np.ascontiguousarray(imgs, dtype=np.uint8)).to(device)
    return DeviceImageLoader(images, torch.as_tensor(labels, dtype=torch.int64).to(device), batch_size, aug,
                             shuffle=shuffle, drop_last=drop_last, seed=seed, rank=rank, world_size=world_size,
                             length=length)


from torchbooster_amd.data.readers import (CIFARBinaryDataset, ImageFolderDataset, MNISTDataset,  # noqa: E402
                                           pack_folder)
