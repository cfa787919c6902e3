"""Readers for the reference's own data sources: MNIST idx files, CIFAR-10 /
CIFAR-100 binary batches, image folders, and the streaming folder -> LMDB packer -- on tiny
fixtures written here in each on-disk format, resolved through ``DatasetConfig.make`` exactly as
the reference's YAMLs name them (/root/reference/torchbooster/config.py:567-576: ``root/<split>``,
``torchvision.datasets.<NAME>``; COCO / paintings ``ImageFolder``s, examples/img_stt/online/
online.py:78-82, adain/adain.py:72-94)."""
import gzip
import os
import struct
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from torchbooster_amd.config import DatasetConfig
from torchbooster_amd.data import (CIFARBinaryDataset, ImageFolderDataset, LMDBImageDataset, MNISTDataset,
                                   pack_folder)
from torchbooster_amd.data.readers import load_image, read_idx
from torchbooster_amd.dataset import Split

ROOT = Path(__file__).resolve().parents[1]


def _idx(path, arr, gz=False):
    code = {np.uint8: 0x08}[arr.dtype.type]
    hdr = bytes([0, 0, code, arr.ndim]) + struct.pack(">" + "I" * arr.ndim, *arr.shape)
    data = hdr + arr.tobytes()
    if gz:
        with gzip.open(str(path) + ".gz", "wb") as f:
            f.write(data)
    else:
        Path(path).write_bytes(data)


def _mnist(root, n_train=7, n_test=3, gz=False):
    rng = np.random.default_rng(0)
    raw = Path(root) / "MNIST" / "raw"  # torchvision's layout under root/<split>
    raw.mkdir(parents=True)
    out = {}
    for pre, n in (("train", n_train), ("t10k", n_test)):
        img = rng.integers(0, 256, (n, 28, 28), dtype=np.uint8)
        lab = rng.integers(0, 10, n, dtype=np.uint8)
        _idx(raw / f"{pre}-images-idx3-ubyte", img, gz)
        _idx(raw / f"{pre}-labels-idx1-ubyte", lab, gz)
        out[pre] = (img, lab)
    return out


@pytest.mark.parametrize("gz", [False, True])
def test_mnist_idx_through_dataset_config(tmp_path, gz):
    ref = {}
    for split in ("train", "test"):
        ref[split] = _mnist(tmp_path / split, gz=gz)
    conf = DatasetConfig(name="mnist", root=str(tmp_path))
    tr = conf.make(Split.TRAIN)
    te = conf.make(Split.TEST)
    assert isinstance(tr, MNISTDataset) and isinstance(te, MNISTDataset)
    assert len(tr) == 7 and len(te) == 3
    img, lab = ref["train"]["train"]
    x, y = tr[4]
    assert x.shape == (1, 28, 28) and x.dtype == torch.float32
    assert torch.equal(x, torch.from_numpy(img[4]).float().unsqueeze(0) / 255.0) and y == int(lab[4])
    timg, tlab = ref["test"]["t10k"]
    x, y = te[2]
    assert torch.equal(x, torch.from_numpy(timg[2]).float().unsqueeze(0) / 255.0) and y == int(tlab[2])
    a, b = tr.arrays_u8()
    assert a.shape == (7, 28, 28, 1) and (b == lab).all()


def test_mnist_transform_and_flat_layout(tmp_path):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (4, 28, 28), dtype=np.uint8)
    _idx(tmp_path / "train-images-idx3-ubyte", img)
    _idx(tmp_path / "train-labels-idx1-ubyte", np.arange(4, dtype=np.uint8))
    ds = MNISTDataset(str(tmp_path), True, transform=lambda t: t * 2)
    assert torch.equal(ds[3][0], torch.from_numpy(img[3]).float().unsqueeze(0) / 255.0 * 2)
    with pytest.raises(ValueError):
        (tmp_path / "bad").write_bytes(b"\x01\x02\x03")
        read_idx(str(tmp_path / "bad"))


def _cifar10(root, n_per=4, n_test=5):
    rng = np.random.default_rng(2)
    d = Path(root) / "cifar-10-batches-bin"
    d.mkdir(parents=True)
    chw = {}
    for name, n in [(f"data_batch_{i}.bin", n_per) for i in range(1, 6)] + [("test_batch.bin", n_test)]:
        lab = rng.integers(0, 10, n, dtype=np.uint8)
        img = rng.integers(0, 256, (n, 3, 32, 32), dtype=np.uint8)
        rec = np.concatenate([lab[:, None], img.reshape(n, -1)], 1)
        (d / name).write_bytes(rec.tobytes())
        chw[name] = (img, lab)
    return chw


def test_cifar10_binary_through_dataset_config(tmp_path):
    ref = _cifar10(tmp_path / "train")
    _cifar10(tmp_path / "test")
    conf = DatasetConfig(name="cifar10", root=str(tmp_path))
    tr = conf.make(Split.TRAIN)
    assert isinstance(tr, CIFARBinaryDataset) and len(tr) == 20
    img, lab = ref["data_batch_3.bin"]
    x, y = tr[2 * 4 + 1]  # third batch, second record
    assert x.shape == (3, 32, 32)
    assert torch.equal(x, torch.from_numpy(img[1]).float() / 255.0) and y == int(lab[1])
    hwc, labels = tr.arrays_u8()
    assert hwc.shape == (20, 32, 32, 3) and np.array_equal(hwc[9], img[1].transpose(1, 2, 0))
    te = conf.make(Split.TEST)
    assert len(te) == 5


def test_cifar100_binary_fine_labels(tmp_path):
    d = tmp_path / "cifar-100-binary"
    d.mkdir()
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (6, 3072), dtype=np.uint8)
    coarse, fine = np.arange(6, dtype=np.uint8), np.arange(50, 56, dtype=np.uint8)
    (d / "train.bin").write_bytes(np.concatenate([coarse[:, None], fine[:, None], img], 1).tobytes())
    ds = CIFARBinaryDataset(str(tmp_path), "cifar100", True)
    assert [ds[i][1] for i in range(6)] == list(range(50, 56))
    (d / "test.bin").write_bytes(b"\x00" * 100)  # not a whole record
    with pytest.raises(ValueError):
        CIFARBinaryDataset(str(tmp_path), "cifar100", False)


def _folder(root, sizes=((40, 56), (64, 48), (33, 33), (70, 90)), classes=("cats", "dogs")):
    from PIL import Image

    rng = np.random.default_rng(4)
    paths = []
    for i, (h, w) in enumerate(sizes):
        c = classes[i % len(classes)]
        (Path(root) / c).mkdir(parents=True, exist_ok=True)
        p = Path(root) / c / f"im{i:02d}.png"
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(p)
        paths.append((str(p), classes.index(c)))
    return paths


def test_image_folder_layout_and_center_crop(tmp_path):
    from PIL import Image

    _folder(tmp_path / "coco")
    ds = ImageFolderDataset(str(tmp_path / "coco"), size=32)
    assert ds.classes == ["cats", "dogs"] and len(ds) == 4
    assert sorted(ds.targets) == [0, 0, 1, 1]
    for i in range(len(ds)):
        x, y = ds[i]
        assert x.shape == (3, 32, 32) and 0.0 <= float(x.min()) and float(x.max()) <= 1.0
        path = ds.samples[i][0]
        with Image.open(path) as im:  # T.Resize(32) + T.CenterCrop(32), by hand
            im = im.convert("RGB")
            w, h = im.size
            s = 32 / min(w, h)
            nw, nh = max(32, round(w * s)), max(32, round(h * s))
            im = im.resize((nw, nh), Image.BILINEAR) if (nw, nh) != (w, h) else im
            l, t = (nw - 32) // 2, (nh - 32) // 2
            ref = np.asarray(im.crop((l, t, l + 32, t + 32)))
        assert torch.equal(x, torch.from_numpy(ref.copy()).permute(2, 0, 1).float() / 255.0)
    # the reference's YAML names: "coco" with the folder at root (split dir absent -> the root itself)
    got = DatasetConfig(name="coco", root=str(tmp_path / "coco")).make(Split.TRAIN, size=32)
    assert isinstance(got, ImageFolderDataset) and len(got) == 4
    got = DatasetConfig(name=f"folder:{tmp_path / 'coco'}", root="/nonexistent").make(Split.TRAIN, size=16)
    assert got[0][0].shape == (3, 16, 16)


def test_flat_image_folder_is_one_class(tmp_path):
    from PIL import Image

    for i in range(3):
        Image.fromarray(np.full((20, 20, 3), 40 * i, np.uint8)).save(tmp_path / f"{i}.jpg")
    ds = ImageFolderDataset(str(tmp_path), size=None)
    assert len(ds) == 3 and set(ds.targets) == {0} and ds[2][0].shape == (3, 20, 20)


@pytest.mark.parametrize("name", ["coco", "paintings", "folder", "folder:/nonexistent/imgs"])
def test_missing_folder_is_fatal_unless_synthetic_requested(tmp_path, caplog, monkeypatch, name):
    """A missing image folder ends the run like the reference's missing dataset
    (logging.fatal + exit(1), /root/reference/torchbooster/config.py:616-617); synthetic
    COCO-shaped data only when TBAMD_SYNTHETIC_DATA=1 asks for it, announced loudly."""
    import logging

    monkeypatch.delenv("TBAMD_SYNTHETIC_DATA", raising=False)
    monkeypatch.setenv("TBAMD_SYNTHETIC_LEN", "8")
    with caplog.at_level(logging.CRITICAL):
        with pytest.raises(SystemExit) as e:
            DatasetConfig(name=name, root=str(tmp_path / "nope")).make(Split.TRAIN)
    assert e.value.code == 1 and "Could not find dataset" in caplog.text
    caplog.clear()
    monkeypatch.setenv("TBAMD_SYNTHETIC_DATA", "1")
    with caplog.at_level(logging.WARNING):
        ds = DatasetConfig(name=name, root=str(tmp_path / "nope")).make(Split.TRAIN)
    assert "SYNTHETIC" in caplog.text and len(ds) == 8


def test_pack_folder_streams_to_lmdb(tmp_path):
    n = 23  # > 10 images: LMDB keys ("0", "1", "10", ...) are written out of numeric order
    from PIL import Image

    rng = np.random.default_rng(5)
    for i in range(n):
        d = tmp_path / "src" / ("a" if i % 3 else "b")
        d.mkdir(parents=True, exist_ok=True)
        Image.fromarray(rng.integers(0, 255, (30 + i, 40, 3), dtype=np.uint8)).save(d / f"{i:03d}.png")
    got = pack_folder(str(tmp_path / "src"), str(tmp_path / "db"), size=24, threads=3)
    assert got == n
    ds = LMDBImageDataset(str(tmp_path / "db"))
    src = ImageFolderDataset(str(tmp_path / "src"), size=24)
    assert len(ds) == n and ds.shape == (24, 24, 3)
    for i in (0, 1, 10, 22):
        x, y = ds[i]
        ref = load_image(src.samples[i][0], 24)
        assert y == src.samples[i][1]
        assert torch.equal(x, torch.from_numpy(ref).permute(2, 0, 1).float() / 255.0)
    # the native multi-threaded fixed-size record gather of the pinned prefetcher reads it
    out = torch.empty(4, ds.record_bytes, dtype=torch.uint8)
    ds.lmdb_reader.gather([3, 0, 22, 11], out, 2)
    assert struct.unpack_from("<q", out[2].numpy().tobytes(), 0)[0] == src.samples[22][1]
    # resolved by name: an LMDB at root/<split> wins
    (tmp_path / "db2").mkdir()
    os.replace(tmp_path / "db" / "data.mdb", tmp_path / "db2" / "data.mdb")
    (tmp_path / "root").mkdir()
    os.replace(tmp_path / "db2", tmp_path / "root" / "train")
    assert isinstance(DatasetConfig(name="coco", root=str(tmp_path / "root")).make(Split.TRAIN), LMDBImageDataset)


def test_online_example_trains_from_an_image_folder(tmp_path):
    """online.py trains 3 iterations from a 4-image folder (no synthetic data) and writes its preview."""
    _folder(tmp_path / "coco")
    base = ROOT / "examples" / "img_stt" / "online" / "online.yml"
    cfg = tmp_path / "conf.yml"
    cfg.write_text(f"#include {base}\nsize: 32\npreview_every: 1\nenv:\n  n_gpu: 0\ndataset:\n  name: coco\n"
                   f"  root: {tmp_path / 'coco'}\nloader:\n  batch_size: 2\n  num_workers: 0\n  drop_last: true\n")
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="3", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    env.pop("TBAMD_SYNTHETIC_DATA", None)
    r = subprocess.run([sys.executable, str(ROOT / "examples" / "img_stt" / "online" / "online.py")], env=env,
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "SYNTHETIC" not in r.stderr
    previews = sorted((tmp_path / "online_previews").iterdir())
    assert len(previews) == 3 and (tmp_path / "online_stylised.png").exists()


def test_pooled_device_loader_indexing():
    """A pooled loader (synthetic ImageNet-shape sets keep a resident pool of distinct images)
    walks the full length; sample i maps to pool entry i % pool (host-side order only)."""
    from torchbooster_amd.data import DeviceImageLoader

    imgs = torch.zeros(10, 4, 4, 3, dtype=torch.uint8)
    labels = torch.arange(10)
    ld = DeviceImageLoader(imgs, labels, batch_size=8, shuffle=True, drop_last=True, length=1000)
    assert len(ld) == 125
    order = ld._order()
    assert len(order) == 1000 and sorted(order.tolist()) == list(range(1000))


def test_random_crop_changes_across_epochs(tmp_path):
    """random_crop draws a new crop each time an image comes round again (the seed had
    no epoch term, so the augmentation was frozen with num_workers=0 / persistent workers)."""
    from PIL import Image

    d = tmp_path / "imgs" / "a"
    d.mkdir(parents=True)
    rng = np.random.default_rng(0)
    Image.fromarray(rng.integers(0, 255, (64, 96, 3), dtype=np.uint8)).save(d / "0.png")
    ds = ImageFolderDataset(str(tmp_path / "imgs"), size=None, transform=None, random_crop=True)
    ds.size = 32  # crop 32 of a 64 x 96 image (resize keeps the shorter side at 32... then crops)
    crops = [ds[0][0] for _ in range(6)]
    assert any(not torch.equal(crops[0], c) for c in crops[1:])
    ds2 = ImageFolderDataset(str(tmp_path / "imgs"), size=32, random_crop=True)
    a = ds2[0][0]
    ds3 = ImageFolderDataset(str(tmp_path / "imgs"), size=32, random_crop=True)
    ds3.set_epoch(0)
    assert torch.equal(a, ds3[0][0])  # same epoch, same draw: reproducible
    ds3.set_epoch(1)
    b = ds3[0][0]
    assert b.shape == a.shape
