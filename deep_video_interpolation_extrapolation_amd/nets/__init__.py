"""Model factory: `nets.__dict__[name](args)` as in the reference (nets/__init__.py:1-33)."""
from .conv import Conv2d
from .ExtraNet import ExtraNet
from .HRNet import HRNet
from .VAEHRNet import VAEHRNet
from .InterNet import InterNet
from .vgg import VGG19, my_vgg, vgg19_features
from .disc import (FrameDiscriminator, FrameLocalDiscriminator, FrameSNDiscriminator, FrameSNLocalDiscriminator,
                   ResnetBlock, ResnetSNBlock, SpectralNorm, VideoDiscriminator, VideoLocalDiscriminator,
                   VideoSNDiscriminator, VideoSNLocalDiscriminator)
from .InterGANNet import InterGANNet, channel_softmax
from .UNet import SegEncoder, SepUNet, UNet, double_conv, down, inconv, outconv, up
from .refine import MSResAttnRefine, SRNRefine
from .InterRefineNet import InterRefineNet, InterStage3Net
from .ExtraNet import ExtraRefineNet, ExtraStage3Net
