"""Offline (Gatys) neural style transfer with VGG-19 (reference: examples/img_stt/offline/offline.py).

Optimises the pixels of one 512x512 image against style Grams and content
features taken by forward hooks on ``vgg19().features[i]`` (torchvision
indices).  VGG-19 runs NHWC bf16 on the native conv kernel; the backward is
dgrad-only (frozen weights) — the stride-1 dgrad also runs on the native kernel.
``content_layers: 29`` (a scalar for a list field) loads fine here (A.2 B4).

Inputs / outputs as in the reference (offline.py:104-121): ``style`` / ``content``
are LOCAL image paths (resized + center-cropped to ``size``, ImageNet-normalised;
synthetic noise with a warning when unset -- there is no network for the
reference's URLs), ``weights`` a local torchvision-layout VGG-19 checkpoint
(``torch.load(weights_only=True)``; random init when unset), and the stylised
image is written to ``output`` as a PNG (the reference ``.show()``s it).
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

import torchbooster_amd.utils as utils  # noqa: E402
from common import max_iters, model_dtype, prepare_model, to_input  # noqa: E402
from torchbooster_amd.config import BaseConfig, EnvironementConfig, OptimizerConfig  # noqa: E402
from torchbooster_amd.imageio import denormalize, image_or_synthetic, normalize, save_image  # noqa: E402
from torchbooster_amd.models import load_weights  # noqa: E402
from torchbooster_amd.models.style import gram_matrix_flat, total_variation  # noqa: E402
from torchbooster_amd.models.vgg import vgg19  # noqa: E402


@dataclass
class Config(BaseConfig):
    n_iter: int
    seed: int
    size: int
    style_layers: list(int)
    style_weights: list(float)
    style_weight: float
    content_layers: list(int)
    content_weights: list(float)
    content_weight: float
    tv_weight: float
    env: EnvironementConfig
    optim: OptimizerConfig
    style: str = ""
    content: str = ""
    weights: str = ""
    output: str = "offline_stylised.png"


def transfer(conf, style, content, mixture, vgg, optim):
    feats = {}

    def hook(module, inp, out, layer):
        feats[layer] = out

    for l in set(conf.style_layers + conf.content_layers):
        vgg[l].register_forward_hook(partial(hook, layer=l))
    with torch.no_grad():
        vgg(style)
        s_grams = [gram_matrix_flat(feats[l]).float() for l in conf.style_layers]
        vgg(content)
        c_feats = [feats[l].float() for l in conf.content_layers]
    last = None
    for _ in range(max_iters(conf.n_iter)):
        vgg(mixture.to(style.dtype))
        s_loss = sum(w * (gram_matrix_flat(feats[l]).float() - g).pow(2).mean()
                     for w, l, g in zip(conf.style_weights, conf.style_layers, s_grams))
        c_loss = sum(w * (feats[l].float() - c).pow(2).mean()
                     for w, l, c in zip(conf.content_weights, conf.content_layers, c_feats))
        loss = conf.style_weight * s_loss + conf.content_weight * c_loss + conf.tv_weight * total_variation(mixture)
        utils.step(loss, optim)
        last = loss.detach()
    return mixture, last


def main(conf: Config) -> None:
    net = vgg19()
    if conf.weights:
        load_weights(net, conf.weights, strict=False)
    vgg = utils.freeze(prepare_model(net.features, conf).eval())
    g = torch.Generator().manual_seed(conf.seed)
    content = to_input(normalize(image_or_synthetic(conf.content, conf.size, "content", g)), conf)
    style = to_input(normalize(image_or_synthetic(conf.style, conf.size, "style", g)), conf)
    mixture = content.detach().float().clone().requires_grad_(True)  # f32 pixels, bf16 features
    optim = conf.optim.make([mixture])
    mixture, loss = transfer(conf, style, content, mixture, vgg, optim)
    out = save_image(denormalize(mixture.detach().float()), conf.output, stretch=True)
    print("final loss", float(loss), tuple(mixture.shape), "->", out)


if __name__ == "__main__":
    conf = Config.load(Path(os.environ.get("TBAMD_CONFIG", Path(__file__).with_name("offline.yml"))))
    utils.seed(conf.seed, deterministic=False)
    utils.boost(enable=True)
    main(conf)
