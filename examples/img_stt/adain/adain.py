"""AdaIN arbitrary style transfer (reference: examples/img_stt/adain/adain.py).

Frozen VGG-16 encoder (hooks at [3, 8, 15, 22]), trainable decoder with fused
InstanceNorm+GELU; loss = per-layer mean/std matching (style) + last-layer MSE
(content).  Two infinite loaders via ``utils.iter_loader``.  Datasets are local
image folders (the reference downloads COCO + Oxford paintings; there is no
network here): a missing folder exits 1 like the reference's missing dataset,
unless ``TBAMD_SYNTHETIC_DATA=1`` asks for synthetic stand-ins.  ``weights``:
a local torchvision-layout VGG-16 checkpoint (random init when unset).  Every
``preview_every`` iterations and at the last one a [style | content | stylised]
grid is written under ``preview_dir`` (the reference ``.show()``s it,
adain.py:160-163).
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass
from functools import partial
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
sys.path.insert(0, str(Path(__file__).resolve().parents[3]))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import torchbooster_amd.distributed as dist  # noqa: E402
import torchbooster_amd.utils as utils  # noqa: E402
from common import max_iters, prepare_model, to_input  # noqa: E402
from torchbooster_amd.config import (BaseConfig, DatasetConfig, EnvironementConfig, LoaderConfig,  # noqa: E402
                                     OptimizerConfig, SchedulerConfig)
from torchbooster_amd.dataset import Split  # noqa: E402
from torchbooster_amd.imageio import denormalize, normalize, save_image  # noqa: E402
from torchbooster_amd.models import load_weights  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.models.style import AdaINDecoder, adain, style_stats_loss  # noqa: E402
from torchbooster_amd.models.vgg import vgg16  # noqa: E402


@dataclass
class Config(BaseConfig):
    n_iter: int
    seed: int
    size: int
    clip: float
    layers: list(int)
    style_weight: float
    content_weight: float
    coco: DatasetConfig
    paintings: DatasetConfig
    env: EnvironementConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    weights: str = ""
    preview_every: int = 500
    preview_dir: str = "adain_previews"


def main(conf: Config) -> None:
    # image folders (the reference's paintings / COCO ImageFolders, adain.py:72-94; missing folders exit 1 unless TBAMD_SYNTHETIC_DATA=1)
    s_loader = conf.loader.make(conf.paintings.make(Split.TRAIN, size=conf.size), shuffle=True,
                                distributed=conf.env.distributed)
    c_loader = conf.loader.make(conf.coco.make(Split.TRAIN, size=conf.size), shuffle=True,
                                distributed=conf.env.distributed)
    vgg = vgg16()
    if conf.weights:
        load_weights(vgg, conf.weights, strict=False)
    encoder = utils.freeze(prepare_model(vgg.features[: max(conf.layers) + 1], conf).eval())
    decoder = prepare_model(AdaINDecoder(), conf)
    optim = conf.optim.make(decoder.parameters())
    sched = conf.scheduler.make(optim)
    feats = {}
    for l in set(conf.layers):
        encoder[l].register_forward_hook(partial(lambda m, i, o, layer: feats.__setitem__(layer, o), layer=l))

    def s_crit(mfs, sfs):
        # == the sum of mse(mu_std(m), mu_std(s)) over the expanded tensors (reference adain.py:134),
        # computed on the [N, C] statistics without materialising the broadcasts
        return style_stats_loss(mfs, sfs)

    s_batches, c_batches = utils.iter_loader(s_loader), utils.iter_loader(c_loader)
    run = RunningAverage()
    n_iter = max_iters(conf.n_iter)
    for it in range(n_iter):
        _, (style, _) = next(s_batches)
        _, (content, _) = next(c_batches)
        # the reference's ctransform ends in Normalize (adain.py:170)
        style, content = to_input(normalize(style), conf), to_input(normalize(content), conf)
        with torch.no_grad():
            encoder(style)
            s_feats = [feats[l].detach() for l in conf.layers]
            encoder(content)
            c_feats = [feats[l].detach() for l in conf.layers]
        mixture = decoder(adain(s_feats[-1], c_feats[-1]))
        encoder(mixture)
        m_feats = [feats[l] for l in conf.layers]
        loss = conf.style_weight * s_crit(m_feats, s_feats) + \
            conf.content_weight * F.mse_loss(m_feats[-1].float(), c_feats[-1].float())
        utils.step(loss, optim, sched, clip=conf.clip)
        run.update(loss.detach())
        if (conf.preview_every > 0 and (it % conf.preview_every == 0 or it == n_iter - 1)
                and dist.is_primary()):
            grid = torch.cat((style[:1], content[:1], mixture[:1].detach()), 0).float()
            save_image(denormalize(grid), Path(conf.preview_dir, f"preview_{it:06d}.png"), nrow=1)
    if dist.is_primary():
        print("mean loss", run.value)


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("adain.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
