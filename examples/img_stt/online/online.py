"""Online (Johnson) fast style transfer (reference: examples/img_stt/online/online.py).

Trains :class:`StyleNet` (weight-tied residual x5, fused InstanceNorm+GELU)
against a frozen VGG-16 loss network; style Grams are precomputed once.
``utils.seed(..., deterministic=False)`` works (A.2 B5).

Inputs / outputs as in the reference (online.py:160-176,190): ``style`` and
``content`` are LOCAL image paths (ImageNet-normalised; synthetic with a warning
when unset -- no network for the reference's URLs), ``weights`` a local
torchvision-layout VGG-16 checkpoint (random init when unset); every
``preview_every`` iterations a [content | stylised] grid is written under
``preview_dir`` (the reference ``.show()``s it), and the stylised ``content``
image is written to ``output`` at the end.  The COCO training set is the
``dataset`` config (``synthetic:coco`` here: no network).
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
from torchbooster_amd.imageio import denormalize, image_or_synthetic, normalize, save_image  # noqa: E402
from torchbooster_amd.models import load_weights  # noqa: E402
from torchbooster_amd.metrics import RunningAverage  # noqa: E402
from torchbooster_amd.models.style import StyleNet, gram_matrix, total_variation  # noqa: E402
from torchbooster_amd.models.vgg import vgg16  # noqa: E402


@dataclass
class Config(BaseConfig):
    n_iter: int
    seed: int
    size: int
    clip: float
    layers: list(int)
    content_layer: int
    style_weight: float
    content_weight: float
    tv_weight: float
    env: EnvironementConfig
    dataset: DatasetConfig
    loader: LoaderConfig
    optim: OptimizerConfig
    scheduler: SchedulerConfig
    style: str = ""
    content: str = ""
    weights: str = ""
    preview_every: int = 500
    preview_dir: str = "online_previews"
    output: str = "online_stylised.png"


def _stylise(net, x):
    with torch.no_grad():
        was = net.training
        net.eval()
        y = net(x)
        net.train(was)
    return y


def main(conf: Config) -> None:
    # an image folder (the reference's COCO ImageFolder, online.py:78-82; synthetic stand-in when absent)
    data = conf.dataset.make(Split.TRAIN, size=conf.size)
    loader = conf.loader.make(data, shuffle=True, distributed=conf.env.distributed)
    loss_net = vgg16()
    if conf.weights:
        load_weights(loss_net, conf.weights, strict=False)
    vgg = utils.freeze(prepare_model(loss_net.features, conf).eval())
    net = prepare_model(StyleNet(), conf)
    optim = conf.optim.make(net.parameters())
    sched = conf.scheduler.make(optim)
    feats = {}
    for l in set(conf.layers + [conf.content_layer]):
        vgg[l].register_forward_hook(partial(lambda m, i, o, layer: feats.__setitem__(layer, o), layer=l))
    g = torch.Generator().manual_seed(conf.seed)
    style = to_input(normalize(image_or_synthetic(conf.style, conf.size, "style", g)), conf)
    preview = to_input(normalize(image_or_synthetic(conf.content, conf.size, "content", g)), conf)
    with torch.no_grad():
        vgg(style)
        s_grams = [gram_matrix(feats[l]).float() for l in conf.layers]
    run = RunningAverage()
    batches = utils.iter_loader(loader)
    for it in range(max_iters(conf.n_iter)):
        _, (content, _) = next(batches)
        content = to_input(normalize(content), conf)  # the reference's ctransform ends in Normalize
        if content.shape[-1] != conf.size:
            content = F.interpolate(content, size=(conf.size, conf.size))
        with torch.no_grad():
            vgg(content)
            c_feat = feats[conf.content_layer].float()
        mixture = net(content)
        vgg(mixture)
        m_grams = [gram_matrix(feats[l]).float() for l in conf.layers]
        s_loss = sum(F.mse_loss(m, s.expand_as(m)) for m, s in zip(m_grams, s_grams))
        c_loss = F.mse_loss(feats[conf.content_layer].float(), c_feat)
        loss = conf.style_weight * s_loss + conf.content_weight * c_loss + \
            conf.tv_weight * total_variation(mixture.float())
        utils.step(loss, optim, sched, clip=conf.clip)
        run.update(loss.detach())
        if conf.preview_every > 0 and it % conf.preview_every == 0 and dist.is_primary():
            grid = torch.cat((preview, _stylise(net, preview)), 0).float()
            save_image(denormalize(grid), Path(conf.preview_dir, f"preview_{it:06d}.png"), stretch=True, nrow=1)
    if dist.is_primary():
        out = save_image(denormalize(_stylise(net, preview).float()), conf.output, stretch=True)
        print("mean loss", run.value, "->", out)


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("online.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    dist.launch(main, conf.env.n_gpu, conf.env.n_machine, conf.env.machine_rank, conf.env.dist_url, args=(conf,))
