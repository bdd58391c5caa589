"""Offline stand-ins for the reference's missing third-party modules (fixture generation
only; never shipped, never imported by the product or by tests at run time).

The reference (lzhangbj/deep_video_interpolation_extrapolation) imports yacs, torchvision
0.2.2, tensorboardX and cv2, none of which are installed here, and `np.int` (removed in
numpy >= 1.24).  These stubs provide exactly what the hot path touches:
  * yacs.config.CfgNode          -> attribute dict (nets/HRNet.py:236)
  * torchvision.models.vgg19()   -> VGG19 `features` layout with the deterministic
                                    synthetic weights of oracle/vgg_synth.py (pretrained
                                    ImageNet weights need a network fetch)
  * torchvision.utils/transforms/datasets, tensorboardX, cv2 -> no-ops
  * F.grid_sample                -> align_corners=True default (torch 1.0.1 semantics, fyp.yml:125)
"""
import sys
import types

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

REF = "/root/reference"


def install(vgg_state_fn):
    if not hasattr(np, "int"):
        np.int = int
    yacs = types.ModuleType("yacs")
    cfg = types.ModuleType("yacs.config")

    class CfgNode(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    cfg.CfgNode = CfgNode
    yacs.config = cfg
    sys.modules["yacs"] = yacs
    sys.modules["yacs.config"] = cfg

    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")

    class _VGG(nn.Module):
        def __init__(self):
            super().__init__()
            cfgl = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
            layers, cin = [], 3
            for v in cfgl:
                if v == "M":
                    layers.append(nn.MaxPool2d(2, 2))
                else:
                    layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
                    cin = v
            self.features = nn.Sequential(*layers)
            with torch.no_grad():
                self.load_state_dict(vgg_state_fn(), strict=False)

    def vgg19(pretrained=False, **kw):
        return _VGG()

    def resnet101(pretrained=False, **kw):
        raise RuntimeError("resnet101 weights unavailable offline")

    models.vgg19 = vgg19
    models.resnet101 = resnet101
    tv.models = models
    utils = types.ModuleType("torchvision.utils")
    utils.make_grid = lambda *a, **k: None
    utils.save_image = lambda *a, **k: None
    tv.utils = utils
    transforms = types.ModuleType("torchvision.transforms")

    class _Any:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x, *a, **k):
            return x

    for n in ("Compose", "RandomCrop", "Resize", "ToTensor", "Normalize", "CenterCrop", "RandomHorizontalFlip"):
        setattr(transforms, n, _Any)
    tv.transforms = transforms
    datasets = types.ModuleType("torchvision.datasets")
    tv.datasets = datasets
    for name, mod in (("torchvision", tv), ("torchvision.models", models), ("torchvision.utils", utils),
                      ("torchvision.transforms", transforms), ("torchvision.datasets", datasets)):
        sys.modules[name] = mod
    tbx = types.ModuleType("tensorboardX")

    class SummaryWriter:
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, k):
            return lambda *a, **kw: None

    tbx.SummaryWriter = SummaryWriter
    sys.modules["tensorboardX"] = tbx
    sys.modules["cv2"] = types.ModuleType("cv2")

    _gs = F.grid_sample

    def grid_sample(input, grid, mode="bilinear", padding_mode="zeros", align_corners=True):
        return _gs(input, grid, mode=mode, padding_mode=padding_mode, align_corners=align_corners)

    F.grid_sample = grid_sample
    if REF not in sys.path:
        sys.path.insert(0, REF)
