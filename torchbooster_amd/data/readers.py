"""Readers for the reference's own data sources, with no torchvision in the stack.

The reference resolves ``DatasetConfig(name="mnist" | "cifar10")`` through
``torchvision.datasets.<NAME>(root/<split>, train=...)`` (/root/reference/torchbooster/config.py:571-576,
picked by lenet.yml:8-9, resnet.yml:10-11, gan.yml:11-12, vae.yml:12-13) and trains the style-transfer
examples on image folders (COCO / painting ``ImageFolder``s: /root/reference/examples/img_stt/online/
online.py:78-82, adain/adain.py:72-94).  Here:

* :class:`MNISTDataset` reads the idx files (``train-images-idx3-ubyte`` / ``t10k-...``, optionally
  ``.gz``) from the torchvision layout ``<root>/MNIST/raw/`` or flat in ``<root>`` (also
  Fashion-MNIST / KMNIST files, which share the format);
* :class:`CIFARBinaryDataset` reads the CIFAR-10 / CIFAR-100 **binary** batches
  (``cifar-10-batches-bin/data_batch_{1..5}.bin`` / ``test_batch.bin``; ``cifar-100-binary/train.bin`` /
  ``test.bin``) -- never the pickled python batches;
* :class:`ImageFolderDataset` is ``ImageFolder``: one class per sub-directory (sorted), PIL decode
  in the loader workers, shorter-side resize + center or random crop;
* :func:`pack_folder` streams an image folder into an LMDB of fixed-size uint8 records
  (the :class:`~torchbooster_amd.data.LMDBImageDataset` format, read by the native pinned prefetcher)
  through the native streaming writer (csrc/lmdb_core.cpp ``LmdbStreamWriter``): one image in memory per
  worker, never the whole set.

Every map-style reader returns what ``ToTensor`` would give the reference's transform -- a float CHW
tensor in [0, 1] -- and applies ``transform`` to it; ``arrays_u8()`` exposes the whole (small) set as
uint8 NHWC for the device-resident loader (data/__init__.py ``device_loader``).
"""
from __future__ import annotations

import gzip
import os
import struct
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

__all__ = ["MNISTDataset", "CIFARBinaryDataset", "ImageFolderDataset", "pack_folder", "find_mnist",
           "find_cifar", "IMG_EXTENSIONS", "load_image"]

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


# --------------------------------------------------------------------------- MNIST idx
def _open(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_idx(path: str) -> np.ndarray:
    """An idx file (``0x0000`` + dtype byte + ndim byte, big-endian dims, then the data)."""
    with _open(path) as f:
        raw = f.read()
    if len(raw) < 4 or raw[0] != 0 or raw[1] != 0:
        raise ValueError(f"{path}: not an idx file")
    types = {0x08: np.uint8, 0x09: np.int8, 0x0B: ">i2", 0x0C: ">i4", 0x0D: ">f4", 0x0E: ">f8"}
    if raw[2] not in types:
        raise ValueError(f"{path}: unknown idx dtype 0x{raw[2]:02x}")
    nd = raw[3]
    dims = struct.unpack_from(">" + "I" * nd, raw, 4)
    dt = np.dtype(types[raw[2]])
    off = 4 + 4 * nd
    n = int(np.prod(dims)) if dims else 1
    if len(raw) < off + n * dt.itemsize:
        raise ValueError(f"{path}: truncated ({len(raw)} bytes for dims {dims})")
    return np.frombuffer(raw, dtype=dt, count=n, offset=off).reshape(dims).astype(dt.newbyteorder("="))


def _first(root: str, names: Sequence[str]) -> Optional[str]:
    for d in (os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw"), root):
        for n in names:
            for ext in ("", ".gz"):
                p = os.path.join(d, n + ext)
                if os.path.isfile(p):
                    return p
    return None


def find_mnist(root: str, train: bool) -> Optional[Tuple[str, str]]:
    """(images, labels) idx paths under ``root`` (torchvision layout or flat), or None."""
    pre = "train" if train else "t10k"
    img = _first(root, [f"{pre}-images-idx3-ubyte", f"{pre}-images.idx3-ubyte"])
    lab = _first(root, [f"{pre}-labels-idx1-ubyte", f"{pre}-labels.idx1-ubyte"])
    return (img, lab) if img and lab else None


class MNISTDataset(Dataset):
    """MNIST from its idx files: item ``i`` = (float [1, 28, 28] in [0, 1], int label)."""

    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None) -> None:
        paths = find_mnist(root, train)
        if paths is None:
            raise FileNotFoundError(f"no MNIST idx files under {root}")
        self.data = read_idx(paths[0])  # [N, 28, 28] uint8 (torchvision's .data)
        self.targets = read_idx(paths[1]).astype(np.int64)
        if self.data.ndim != 3 or len(self.data) != len(self.targets):
            raise ValueError(f"MNIST idx shapes {self.data.shape} / {self.targets.shape} do not match")
        self.transform = transform
        self.train = train

    def __len__(self) -> int:
        return len(self.targets)

    def arrays_u8(self):
        return self.data[..., None], self.targets

    def __getitem__(self, i: int):
        x = torch.from_numpy(np.array(self.data[i], copy=True)).unsqueeze(0).float().div_(255.0)
        if self.transform is not None:
            x = self.transform(x)
        return x, int(self.targets[i])


# --------------------------------------------------------------------------- CIFAR binary
_CIFAR = {
    "cifar10": ("cifar-10-batches-bin", [f"data_batch_{i}.bin" for i in range(1, 6)], ["test_batch.bin"], 1),
    "cifar100": ("cifar-100-binary", ["train.bin"], ["test.bin"], 2),
}


def find_cifar(root: str, name: str, train: bool) -> Optional[List[str]]:
    sub, tr, te, _ = _CIFAR[name]
    for d in (os.path.join(root, sub), root):
        files = [os.path.join(d, f) for f in (tr if train else te)]
        if all(os.path.isfile(f) for f in files):
            return files
    return None


class CIFARBinaryDataset(Dataset):
    """CIFAR-10 / CIFAR-100 binary batches: records of ``<label byte(s)><3072 bytes CHW>``
    (CIFAR-100: coarse then fine label; the fine label is the target, like torchvision).
    Item ``i`` = (float [3, 32, 32] in [0, 1], int label)."""

    def __init__(self, root: str, name: str = "cifar10", train: bool = True,
                 transform: Optional[Callable] = None) -> None:
        name = name.lower()
        if name not in _CIFAR:
            raise ValueError(f"unknown CIFAR variant {name}")
        files = find_cifar(root, name, train)
        if files is None:
            raise FileNotFoundError(f"no {name} binary batches under {root}")
        nlab = _CIFAR[name][3]
        rec = nlab + 3 * 32 * 32
        parts = []
        for f in files:
            raw = np.fromfile(f, dtype=np.uint8)
            if raw.size % rec:
                raise ValueError(f"{f}: {raw.size} bytes is not a whole number of {rec}-byte records")
            parts.append(raw.reshape(-1, rec))
        arr = np.concatenate(parts)
        self.targets = arr[:, nlab - 1].astype(np.int64)
        # NHWC uint8 (torchvision's .data layout)
        self.data = np.ascontiguousarray(arr[:, nlab:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
        self.transform = transform
        self.train = train

    def __len__(self) -> int:
        return len(self.targets)

    def arrays_u8(self):
        return self.data, self.targets

    def __getitem__(self, i: int):
        x = torch.from_numpy(np.array(self.data[i], copy=True)).permute(2, 0, 1).float().div_(255.0)
        if self.transform is not None:
            x = self.transform(x)
        return x, int(self.targets[i])


# --------------------------------------------------------------------------- image folders
def load_image(path: str, size: Optional[int] = None, crop: str = "center",
               rng: Optional[np.random.Generator] = None) -> np.ndarray:
    """Decode ``path`` to uint8 RGB HWC; ``size``: shorter side resized to ``size`` (bilinear,
    like ``T.Resize(size)``), then a ``size`` x ``size`` crop (``"center"`` or ``"random"``)."""
    from PIL import Image

    with Image.open(path) as im:
        im = im.convert("RGB")
        if size is not None:
            w, h = im.size
            s = size / min(w, h)
            nw, nh = max(size, round(w * s)), max(size, round(h * s))
            if (nw, nh) != (w, h):
                im = im.resize((nw, nh), Image.BILINEAR)
            if crop == "random":
                g = rng if rng is not None else np.random.default_rng()
                x0, y0 = int(g.integers(0, nw - size + 1)), int(g.integers(0, nh - size + 1))
            else:
                x0, y0 = (nw - size) // 2, (nh - size) // 2
            im = im.crop((x0, y0, x0 + size, y0 + size))
        return np.asarray(im, dtype=np.uint8).copy()


def _scan(root: str, flat_ok: bool = True) -> Tuple[List[Tuple[str, int]], List[str]]:
    classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
    samples: List[Tuple[str, int]] = []
    for ci, c in enumerate(classes):
        for dp, _, fs in sorted(os.walk(os.path.join(root, c), followlinks=True)):
            samples.extend((os.path.join(dp, f), ci) for f in sorted(fs) if f.lower().endswith(IMG_EXTENSIONS))
    if not samples and flat_ok:  # a flat folder of images: one class
        samples = [(os.path.join(root, f), 0) for f in sorted(os.listdir(root)) if f.lower().endswith(IMG_EXTENSIONS)]
        classes = ["."] if samples else []
    return samples, classes


class ImageFolderDataset(Dataset):
    """``torchvision.datasets.ImageFolder`` semantics: ``root/<class>/**/<image>`` with classes
    sorted by name (a flat folder of images is one class).  Item ``i`` = (float [3, size, size] in
    [0, 1], class index); images are decoded with PIL when the item is read (in the DataLoader
    workers), resized on the shorter side and center- (or ``random_crop``) cropped to ``size``."""

    def __init__(self, root: str, size: Optional[int] = 256, transform: Optional[Callable] = None,
                 random_crop: bool = False, seed: int = 0) -> None:
        if not os.path.isdir(root):
            raise FileNotFoundError(f"image folder {root} does not exist")
        self.root = root
        self.samples, self.classes = _scan(root)
        if not self.samples:
            raise FileNotFoundError(f"no images ({', '.join(IMG_EXTENSIONS)}) under {root}")
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}
        self.targets = [c for _, c in self.samples]
        self.size, self.transform, self.random_crop, self.seed = size, transform, random_crop, seed
        self.epoch = 0
        self._draws: dict = {}  # index -> times drawn in this process (persistent workers, no workers)

    def set_epoch(self, epoch: int) -> None:
        """Per-epoch random crops (utils.iter_loader calls it; worker copies made after it carry it)."""
        self.epoch = int(epoch)

    def __len__(self) -> int:
        return len(self.samples)

    def __getitem__(self, i: int):
        path, label = self.samples[i]
        rng = None
        if self.random_crop:
            # a fresh crop every time an image comes round again: the epoch (set_epoch) and this
            # process's draw count of the index (persistent workers never see set_epoch)
            k = self._draws.get(i, 0)
            self._draws[i] = k + 1
            rng = np.random.default_rng((self.seed, self.epoch, k, i, os.getpid()))
        img = load_image(path, self.size, "random" if self.random_crop else "center", rng)
        x = torch.from_numpy(img).permute(2, 0, 1).float().div_(255.0)
        if self.transform is not None:
            x = self.transform(x)
        return x, label


def pack_folder(src: str, dst: str, size: int = 256, threads: int = 8, map_size: int = 1 << 30) -> int:
    """Stream the image folder ``src`` (:class:`ImageFolderDataset` layout) into an LMDB at ``dst``
    of ``size`` x ``size`` uint8 RGB records (shorter-side resize + center crop) in the
    :class:`~torchbooster_amd.data.LMDBImageDataset` format (``str(i)`` -> ``<q label><HWC bytes>``,
    ``b"shape"``, ``b"length"``).  Images are decoded ``threads`` at a time and written as they
    arrive, in key order; host memory stays at a few images per thread whatever the folder size.
    Returns the number of images."""
    from torchbooster_amd.ops._ext import native

    samples, _ = _scan(src)
    if not samples:
        raise FileNotFoundError(f"no images under {src}")
    n = len(samples)
    keys = sorted(str(i) for i in range(n))  # LMDB key order: lexicographic ("0", "1", "10", ...)
    if not os.path.splitext(dst)[1]:
        os.makedirs(dst, exist_ok=True)
    w = native().LmdbStreamWriter(str(dst), int(map_size), 4096)

    def rec(k: str) -> bytes:
        path, label = samples[int(k)]
        return struct.pack("<q", label) + load_image(path, size).tobytes()

    with ThreadPoolExecutor(max(1, threads)) as ex:
        win = max(2, 4 * threads)  # bounded look-ahead: at most `win` decoded images in flight
        futs = [ex.submit(rec, k) for k in keys[:win]]
        for j, k in enumerate(keys):
            v = futs[j].result()
            futs[j] = None
            if j + win < n:
                futs.append(ex.submit(rec, keys[j + win]))
            w.add(k.encode(), v)
    w.add(b"length", str(n).encode())
    w.add(b"shape", f"{size},{size},3".encode())
    w.close()
    return n
