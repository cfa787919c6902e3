"""DeviceAugment (CPU reference path) and the LoaderConfig routing on CPU; the
kernel itself is checked against this reference in tests/test_gpu_data.py."""
import numpy as np
import torch

from torchbooster_amd.config import LoaderConfig
from torchbooster_amd.data import DeviceAugment, SyntheticImageDataset


def test_params_ranges_follow_torchvision():
    a = DeviceAugment(size=32, padding=4, hflip=True, rotate=15, randaugment=True)
    p = a.params(4096, 32, 32, np.random.default_rng(0))
    assert p[:, 0].min() == -4 and p[:, 0].max() == 4 and set(np.unique(p[:, 2])) == {0.0, 1.0}
    assert np.abs(p[:, 3]).max() <= 15 and set(np.unique(p[:, 4]).astype(int)) == set(range(14))
    mags = {int(o): abs(float(m)) for o, m in zip(p[:, 4], p[:, 5])}
    assert abs(mags[1] - 0.09) < 1e-6 and abs(mags[5] - 9.0) < 1e-5 and abs(mags[6] - 0.27) < 1e-6
    assert mags[10] == 7 and abs(mags[11] - 178.5) < 1e-4 and abs(mags[3] - 150 / 331 * 32 * 0.3) < 1e-4


def test_reference_ops():
    a = DeviceAugment(mean=(0.0,), std=(1.0,))
    img = np.arange(4 * 4 * 3, dtype=np.uint8).reshape(4, 4, 3) * 5
    ident = a.reference(img, np.zeros(8, np.float32))
    assert np.allclose(ident, img.transpose(2, 0, 1) / 255.0)
    flip = a.reference(img, np.array([0, 0, 1, 0, 0, 0, 0, 0], np.float32))
    assert np.allclose(flip, img[:, ::-1].transpose(2, 0, 1) / 255.0)
    crop = DeviceAugment(size=4, padding=1, mean=(0.0,), std=(1.0,)).reference(
        img, np.array([-1, 1, 0, 0, 0, 0, 0, 0], np.float32))
    assert np.allclose(crop[:, 0, :3], img[1, 1:4].T / 255.0)  # row -1 reflects to row 1
    post = a.reference(img, np.array([0, 0, 0, 0, 10, 7, 0, 0], np.float32))
    assert np.allclose(post, (img & 0xFE).transpose(2, 0, 1) / 255.0)
    sol = a.reference(img, np.array([0, 0, 0, 0, 11, 100, 0, 0], np.float32))
    want = np.where(img >= 100, 255 - img, img)
    assert np.allclose(sol, want.transpose(2, 0, 1) / 255.0)
    eq = a.reference(img, np.array([0, 0, 0, 0, 13, 0, 0, 0], np.float32))
    assert eq.shape == (3, 4, 4) and eq.max() <= 1.0


def test_loader_config_cpu_keeps_dataloader_and_applies_transform():
    ds = SyntheticImageDataset(8, (3, 32, 32), 10, transform=DeviceAugment(size=32, padding=4, hflip=True,
                                                                          randaugment=True))
    loader = LoaderConfig(batch_size=4).make(ds)
    assert isinstance(loader, torch.utils.data.DataLoader)
    x, y = next(iter(loader))
    assert x.shape == (4, 3, 32, 32) and x.dtype == torch.float32
