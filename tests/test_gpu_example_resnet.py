"""The ResNet example on its ImageNet-shape config (examples/img_cls/resnet/resnet50_imagenet.yml,
synthetic data when no ImageNet folder exists) runs through the framework path -- config ->
device loader (a resident pool of distinct synthetic images) -> native model -> utils.step -- and
reports its training throughput (TBAMD_EXAMPLE_TIMING), the figure bench.py's headline is checked
against.  Reference: examples/img_cls/resnet/resnet.py:44-68,111."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pooled_synthetic_device_loader():
    from torchbooster_amd.data import DeviceAugment, SyntheticImageDataset, device_loader

    ds = SyntheticImageDataset(1_281_167, (3, 224, 224), 1000, seed=0, transform=DeviceAugment(hflip=True))
    ld = device_loader(ds, 64, shuffle=True, drop_last=True)
    assert ld is not None and ld.images.shape[0] < 10000 and len(ld) == 1_281_167 // 64
    x, y = next(iter(ld))
    assert x.shape == (64, 3, 224, 224) and x.is_cuda and y.shape == (64,)
    assert int(y.max()) < 1000 and torch.isfinite(x.float()).all()


@pytest.mark.timeout(600)
def test_resnet50_imagenet_example_runs_and_times(tmp_path):
    cfg = tmp_path / "r50.yml"
    inc = os.path.join(ROOT, "examples", "img_cls", "resnet", "resnet50_imagenet.yml")
    cfg.write_text(f"#include {inc}\nenv:\n  fp16: true\n  n_gpu: 1\n  distributed: false\n"
                   "dataset:\n  name: synthetic:imagenet\n  root: /nonexistent/imagenet\n"
                   "loader:\n  batch_size: 64\n  num_workers: 0\n  pin_memory: false\n  drop_last: true\n")
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="8", TBAMD_EXAMPLE_TIMING="3",
               MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "img_cls", "resnet", "resnet.py")], env=env,
                       capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{\"example_img_s\"")]
    assert lines and lines[0]["iters"] == 5 and lines[0]["example_img_s"] > 0, r.stdout[-2000:]
    assert np.isfinite(lines[0]["example_img_s"])
