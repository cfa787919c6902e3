"""Every example runs end-to-end on CPU for a couple of iterations (gloo / in-process),
through the same Config.load -> seed -> boost -> launch -> make -> step pipeline."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EX = ROOT / "examples"

CASES = [
    ("img_cls/lenet/lenet.py", "lenet.yml", "env:\n  n_gpu: 0\nloader:\n  batch_size: 16\n  num_workers: 0\n"),
    ("img_cls/resnet/resnet.py", "resnet.yml",
     "env:\n  n_gpu: 0\nloader:\n  batch_size: 8\n  num_workers: 0\n  drop_last: true\n"),
    ("img_gen/gan/gan.py", "gan.yml", "env:\n  n_gpu: 0\nloader:\n  batch_size: 16\n  num_workers: 0\n"),
    ("img_gen/vae/vae.py", "vae.yml", "env:\n  n_gpu: 0\nloader:\n  batch_size: 16\n  num_workers: 0\n"),
    ("img_gen/dcgan/dcgan.py", "dcgan.yml",
     "width: 8\nenv:\n  n_gpu: 0\nloader:\n  batch_size: 4\n  num_workers: 0\n  drop_last: true\n"),
    ("img_stt/offline/offline.py", "offline.yml", "size: 32\nenv:\n  n_gpu: 0\n"),
    ("img_stt/online/online.py", "online.yml",
     "size: 32\nenv:\n  n_gpu: 0\nloader:\n  batch_size: 2\n  num_workers: 0\n  drop_last: true\n"),
    ("img_stt/adain/adain.py", "adain.yml",
     "size: 32\nenv:\n  n_gpu: 0\nloader:\n  batch_size: 2\n  num_workers: 0\n  drop_last: true\n"),
]


@pytest.mark.parametrize("script,yml,override", CASES, ids=[c[0].split("/")[-1] for c in CASES])
def test_example_runs_on_cpu(tmp_path, script, yml, override):
    base = EX / Path(script).parent / yml
    cfg = tmp_path / "conf.yml"
    cfg.write_text(f"#include {base}\n{override}")
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="2", TBAMD_SYNTHETIC_LEN="64", TBAMD_SYNTHETIC_DATA="1",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, str(EX / script)], env=env, capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    # the examples' products, as the reference shows them (written as PNGs here)
    outs = {"offline.py": ["offline_stylised.png"], "online.py": ["online_stylised.png", "online_previews"],
            "adain.py": ["adain_previews"], "gan.py": ["gan_samples.png"], "vae.py": ["vae_samples.png"],
            "dcgan.py": ["dcgan_samples.png"]}.get(Path(script).name, [])
    for o in outs:
        assert (tmp_path / o).exists(), (o, sorted(p.name for p in tmp_path.iterdir()))


def test_offline_style_transfer_reads_and_writes_pngs(tmp_path):
    """``offline.py`` with two local PNG paths writes the stylised PNG."""
    import numpy as np
    from PIL import Image

    rng = np.random.default_rng(0)
    for name in ("style.png", "content.png"):
        Image.fromarray(rng.integers(0, 255, (40, 56, 3), dtype=np.uint8)).save(tmp_path / name)
    base = EX / "img_stt" / "offline" / "offline.yml"
    cfg = tmp_path / "conf.yml"
    cfg.write_text(f"#include {base}\nsize: 32\nstyle: {tmp_path / 'style.png'}\ncontent: {tmp_path / 'content.png'}\n"
                   f"output: {tmp_path / 'out' / 'stylised.png'}\nenv:\n  n_gpu: 0\n")
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="2", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, str(EX / "img_stt" / "offline" / "offline.py")], env=env, capture_output=True,
                       text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "synthetic" not in r.stderr  # the configured images were used
    img = Image.open(tmp_path / "out" / "stylised.png")
    assert img.size == (32, 32) and img.mode == "RGB"


def test_vit_example_lmdb_cpu(tmp_path):
    base = EX / "vit" / "vit.yml"
    cfg = tmp_path / "conf.yml"
    cfg.write_text(f"#include {base}\narch: vit_tiny\nimage: 32\nnum_classes: 10\nlmdb: {tmp_path / 'db'}\n"
                   "lmdb_records: 16\nenv:\n  n_gpu: 0\nloader:\n  batch_size: 4\n  num_workers: 0\n"
                   "  drop_last: true\n")
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="2", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, str(EX / "vit" / "vit.py")], env=env, capture_output=True, text=True,
                       timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]


def test_gan_example_ddp_gloo_world2(tmp_path):
    base = EX / "img_gen" / "gan" / "gan.yml"
    cfg = tmp_path / "conf.yml"
    # n_gpu 0 + distributed -> 2 gloo ranks through launch(n_proc=2) is not reachable from YAML;
    # use torchrun-style env:// instead (the driver's launch mode)
    cfg.write_text(f"#include {base}\nenv:\n  n_gpu: 0\n  distributed: true\nloader:\n  batch_size: 8\n"
                   "  num_workers: 0\n")
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="2", TBAMD_SYNTHETIC_LEN="64", TBAMD_SYNTHETIC_DATA="1",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000),
                        str(EX / "img_gen" / "gan" / "gan.py")], env=env, capture_output=True, text=True,
                       timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
