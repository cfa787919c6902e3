"""Model zoo: the reference's example workloads + the north-star configs.

img_cls: ResNet-18/34/50/101/152 (``resnet``), LeNet (``small``);
img_gen: MLP GAN / VAE (``small``), DCGAN-128 (``dcgan``);
img_stt: VGG-16/19 features (``vgg``), StyleNet / AdaIN decoder (``style``);
north-star: ViT-B/16 (``vit``);
torchvision layout from stock modules + local pretrained weights: ``tv`` (``load_weights``).
"""
from torchbooster_amd.models.dcgan import DCGANDiscriminator, DCGANGenerator, dcgan128
from torchbooster_amd.models.resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152
from torchbooster_amd.models.small import VAE, LeNet, MLPDiscriminator, MLPGenerator, lenet
from torchbooster_amd.models.style import AdaINDecoder, StyleNet
from torchbooster_amd.models.vgg import VGG, vgg16, vgg19
from torchbooster_amd.models.vit import ViT, vit_b_16, vit_s_16, vit_tiny
from torchbooster_amd.models import tv
from torchbooster_amd.models.tv import load_weights
