"""Device input pipeline: the augmentation kernel (csrc/data.hip augment_u8_k) against
DeviceAugment.reference (NumPy), and the device loaders behind LoaderConfig.make."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from torchbooster_amd.config import LoaderConfig  # noqa: E402
from torchbooster_amd.data import DeviceAugment, DeviceImageLoader, SyntheticImageDataset  # noqa: E402


@pytest.mark.parametrize("shape", [(32, 32, 3), (28, 28, 1)])
@pytest.mark.parametrize("op", list(range(14)))
def test_augment_kernel_matches_reference(shape, op):
    H, W, C = shape
    rng = np.random.default_rng(op + 100 * C)
    imgs = rng.integers(0, 256, size=(64, H, W, C), dtype=np.uint8)
    imgs[:8] = (imgs[:8] // 64) * 40  # low-contrast images (autocontrast / equalize edge cases)
    a = DeviceAugment(size=(H, W), padding=4, hflip=True, rotate=15, randaugment=True,
                      mean=(0.4914, 0.4822, 0.4465)[:C], std=(0.2023, 0.1994, 0.2010)[:C], dtype=torch.float32)
    p = a.params(64, H, W, rng)
    p[:, 4] = op  # force the first RandAugment op
    sign = np.where(np.arange(64) % 2 == 1, 1.0, -1.0) if op in range(1, 10) else np.ones(64)
    p[:, 5] = [a._ra_mag(op, H, W) * sign[i] for i in range(64)]
    got = a.apply(torch.from_numpy(imgs).cuda(), p).cpu().numpy()
    want = np.stack([a.reference(imgs[i], p[i]) for i in range(64)])
    diff = np.abs(got - want)
    # nearest-neighbour rounding at exact .5 boundaries may pick the other pixel (fma order)
    assert (diff < 1e-4).mean() > 0.995, (op, (diff < 1e-4).mean())
    assert got.shape == (64, C, H, W)


@pytest.mark.parametrize("shape,size,pad", [((32, 32, 3), 32, 4), ((256, 256, 3), 224, 0)])
def test_crop_flip_stream_kernel_matches_reference(shape, size, pad):
    """Geometry-only pipelines (crop + flip, any image size: ImageNet's 224x224x3 does not fit the
    LDS pipeline) run csrc/data.hip crop_flip_u8_k; it must equal the NumPy reference."""
    H, W, C = shape
    rng = np.random.default_rng(7)
    imgs = rng.integers(0, 256, size=(16, H, W, C), dtype=np.uint8)
    a = DeviceAugment(size=size, padding=pad, hflip=True, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                      dtype=torch.float32)
    p = a.params(16, H, W, rng)
    src = torch.arange(15, -1, -1, dtype=torch.int32, device="cuda")
    got = a.apply(torch.from_numpy(imgs).cuda(), p, src).cpu().numpy()
    want = np.stack([a.reference(imgs[15 - i], p[i]) for i in range(16)])
    assert got.shape == (16, C, size, size)
    np.testing.assert_allclose(got, want, atol=1e-5)


def test_device_image_loader_shards_and_epochs():
    ds = SyntheticImageDataset(100, (3, 32, 32), 10, transform=DeviceAugment(size=32, padding=4, hflip=True))
    loader = LoaderConfig(batch_size=16, drop_last=True).make(ds, shuffle=True)
    assert isinstance(loader, DeviceImageLoader) and len(loader) == 6
    x, y = next(iter(loader))
    assert x.is_cuda and x.dtype == torch.bfloat16 and x.shape == (16, 3, 32, 32)
    assert x.is_contiguous(memory_format=torch.channels_last) and y.is_cuda and y.dtype == torch.int64
    first = [yy.cpu() for _, yy in loader]
    loader.set_epoch(1)
    second = [yy.cpu() for _, yy in loader]
    assert not all(torch.equal(a, b) for a, b in zip(first, second))
    # labels follow the images: identity transform reproduces dataset items exactly
    ident = SyntheticImageDataset(10, (3, 8, 8), 10, transform=DeviceAugment(mean=(0.0,), std=(1.0,),
                                                                             dtype=torch.float32))
    ld = LoaderConfig(batch_size=10).make(ident, shuffle=False)
    xb, yb = next(iter(ld))
    for i in range(10):
        xi, yi = SyntheticImageDataset(10, (3, 8, 8), 10)[i]
        assert int(yb[i]) == yi and torch.allclose(xb[i].float().cpu(), xi, atol=1e-6)


def test_pinned_prefetcher_with_augment(tmp_path):
    from torchbooster_amd.data import LMDBImageDataset, PinnedPrefetcher

    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, size=(40, 32, 32, 3), dtype=np.uint8)
    LMDBImageDataset.prepare(tmp_path / "db", imgs, list(range(40)))
    ds = LMDBImageDataset(tmp_path / "db", transform=DeviceAugment(size=32, padding=4, hflip=True,
                                                                   randaugment=True))
    loader = LoaderConfig(batch_size=8, drop_last=True).make(ds, shuffle=True)
    assert isinstance(loader, PinnedPrefetcher)
    n = 0
    for x, y in loader:
        assert x.shape == (8, 3, 32, 32) and x.is_cuda and y.max() < 40
        n += 1
    assert n == 5
