"""Every example runs end-to-end on the GPU (native kernels) for a few iterations:
the same Config.load -> seed -> boost -> launch -> make -> step pipeline as on CPU
(tests/test_examples.py), with ``env.n_gpu: 1`` so models, data and the fused
optimizers live on the MI355X.  Sizes are cut down; each example is one short
child process (sequential, one GPU user at a time)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU collection
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = Path(__file__).resolve().parents[1]
EX = ROOT / "examples"

CASES = [
    ("img_cls/lenet/lenet.py", "lenet.yml", "env:\n  n_gpu: 1\nloader:\n  batch_size: 64\n  num_workers: 0\n"),
    ("img_cls/resnet/resnet.py", "resnet.yml",
     "env:\n  n_gpu: 1\nloader:\n  batch_size: 64\n  num_workers: 0\n  drop_last: true\n"),
    ("img_gen/gan/gan.py", "gan.yml", "env:\n  n_gpu: 1\nloader:\n  batch_size: 64\n  num_workers: 0\n"),
    ("img_gen/vae/vae.py", "vae.yml", "env:\n  n_gpu: 1\nloader:\n  batch_size: 64\n  num_workers: 0\n"),
    ("img_gen/dcgan/dcgan.py", "dcgan.yml",
     "width: 16\nenv:\n  n_gpu: 1\nloader:\n  batch_size: 8\n  num_workers: 0\n  drop_last: true\n"),
    ("img_stt/offline/offline.py", "offline.yml", "size: 64\nenv:\n  n_gpu: 1\n"),
    ("img_stt/online/online.py", "online.yml",
     "size: 64\nenv:\n  n_gpu: 1\nloader:\n  batch_size: 2\n  num_workers: 0\n  drop_last: true\n"),
    ("img_stt/adain/adain.py", "adain.yml",
     "size: 64\nenv:\n  n_gpu: 1\nloader:\n  batch_size: 2\n  num_workers: 0\n  drop_last: true\n"),
]


def _run(script, cfg_text, tmp_path, extra_env=None):
    cfg = tmp_path / "conf.yml"
    cfg.write_text(cfg_text)
    env = dict(os.environ, TBAMD_CONFIG=str(cfg), TBAMD_EXAMPLE_MAX_ITERS="3", TBAMD_SYNTHETIC_LEN="256", TBAMD_SYNTHETIC_DATA="1")
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, str(EX / script)], env=env, capture_output=True, text=True, timeout=110,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r


@pytest.mark.parametrize("script,yml,override", CASES, ids=[c[0].split("/")[-1] for c in CASES])
def test_example_runs_on_gpu(tmp_path, script, yml, override):
    base = EX / Path(script).parent / yml
    _run(script, f"#include {base}\n{override}", tmp_path)


def test_vit_example_lmdb_gpu(tmp_path):
    base = EX / "vit" / "vit.yml"
    _run("vit/vit.py", f"#include {base}\narch: vit_tiny\nimage: 32\nnum_classes: 10\nlmdb: {tmp_path / 'db'}\n"
         "lmdb_records: 64\nenv:\n  n_gpu: 1\nloader:\n  batch_size: 16\n  num_workers: 0\n  drop_last: true\n",
         tmp_path)
