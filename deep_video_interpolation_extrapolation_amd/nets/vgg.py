"""VGG19 perceptual features (reference nets/vgg.py:5-54, `my_vgg`) on the plan engine.

`vgg19_features()` builds torchvision's VGG19 `features` layout (indices 0..36; convs at
0,2,5,7,10,12,14,16,19,21,23,25,28,30,32,34) so a torchvision state_dict loads into it.
The pretrained ImageNet weights of the reference (`vgg19(pretrained=True)`,
losses.py:160,185) need a network fetch; offline they are replaced by a deterministic
synthetic initialisation (private generator, seed 19, kaiming-normal fan-out as in
torchvision's init, zero bias).  Set DVIE_VGG19_WEIGHTS=/path/to/vgg19.pth (a torchvision
state_dict, loaded with weights_only=True) to use real weights.

`my_vgg(vgg)(img)` keeps the reference call signature and returns the five ReLU feature
maps (relu1_2, relu2_2, relu3_4, relu4_4, relu5_4) with 2x2 *average* pooling between
blocks, exactly as the reference wrapper does.
"""
import os

import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import PlanFunction, PlanPool, precision_of
from .conv import Conv2d

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
FEATURE_TAPS = (3, 8, 17, 26, 35)  # ReLU indices returned by my_vgg (x4, x9, x18, x27, x36)
SYNTH_SEED = 19


def synthetic_vgg19_state(seed=SYNTH_SEED):
    """Deterministic stand-in for the ImageNet VGG19 weights ({'features.i.weight': ...})."""
    gen = torch.Generator().manual_seed(seed)
    state = {}
    idx, cin = 0, 3
    for v in VGG19_CFG:
        if v == "M":
            idx += 1
            continue
        std = (2.0 / (v * 9)) ** 0.5
        state[f"features.{idx}.weight"] = torch.randn((v, cin, 3, 3), generator=gen) * std
        state[f"features.{idx}.bias"] = torch.zeros(v)
        cin = v
        idx += 2
    return state


class VGG19(nn.Module):
    def __init__(self, weights=None):
        super().__init__()
        layers = []
        cin = 3
        for v in VGG19_CFG:
            if v == "M":
                layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            else:
                layers += [Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
                cin = v
        self.features = nn.Sequential(*layers)
        if weights is None:
            path = os.environ.get("DVIE_VGG19_WEIGHTS")
            if path:
                sd = torch.load(path, map_location="cpu", weights_only=True)
                weights = {k: v for k, v in sd.items() if k.startswith("features.")}
            else:
                weights = synthetic_vgg19_state()
        self.load_state_dict(weights, strict=False)


def vgg19_features(weights=None):
    return VGG19(weights)


class my_vgg(nn.Module):
    """Reference nets/vgg.py:5-54: five ReLU feature maps, AvgPool2d(2,2) between blocks."""

    sign_log = None  # test support: a list collects the ReLU branches of every loss call, in order

    def __init__(self, vgg):
        super().__init__()
        self.vgg = vgg
        self.avgpool = nn.AvgPool2d(kernel_size=(2, 2), stride=(2, 2))
        self._pool = PlanPool(self._build_plan)
        self.dtype = precision_of()
        for p in self.parameters():
            p.requires_grad = False

    def conv_layers(self):
        return [(i, m) for i, m in enumerate(self.vgg.features) if isinstance(m, nn.Conv2d) and i <= 34]

    def lower(self, g, H, W, normalize, loss=True):
        """Graph: [pred | gt] (2B images) -> features; if loss, the 5 feature-L1 terms."""
        A = L
        inp = g.buffer("vgg_in", H, W, 8)
        g.input_nchw(E.R(inp), "pred", part=0 if loss else None, ext_c=3, normalize=normalize, requires_grad=loss)
        if loss:
            g.input_nchw(E.R(inp), "gt", part=1, ext_c=3, normalize=normalize)
        x = E.R(inp)
        feats = []
        h, w = H, W
        for i, m in enumerate(self.vgg.features):
            if i > 35:
                break
            if isinstance(m, nn.Conv2d):
                b = g.buffer(f"vgg{i}", h, w, m.out_channels)
                g.conv(x, m, E.R(b), act=A.ACT_RELU, trainable=False, name=f"features.{i}")
                x = E.R(b)
                if i + 1 in FEATURE_TAPS:
                    feats.append(x)
                    if loss:
                        g.l1feat(x, weight=1.0 / len(FEATURE_TAPS))
            elif isinstance(m, nn.MaxPool2d) and i < 35:
                h, w = h // 2, w // 2
                b = g.buffer(f"vgg{i}", h, w, x.c)
                g.pool(x, E.R(b))
                x = E.R(b)
        return feats

    def _build_plan(self, key):
        n, H, W, dtype, normalize, loss, dev = key
        g = E.Graph(dtype)
        feats = self.lower(g, H, W, normalize, loss)
        plan = g.compile(2 * n if loss else n, dev, n_bwd=n, backward=loss)
        plan.static_weights = True  # frozen loss network: the weights are packed once
        plan.feats = feats
        return plan

    def invalidate_packs(self):
        """Repack every plan's weights at its next forward.  The packed-weight cache keys on
        (storage, version counter) of the parameters; a write through `p.data` (p.data.copy_,
        a common way to load weights) bumps no version counter, so call this after one."""
        pool = self.__dict__.get("_pool")
        for plans in (pool.plans.values() if pool is not None else ()):
            for p in plans:
                p.invalidate_pack()

    def load_state_dict(self, *args, **kwargs):
        out = super().load_state_dict(*args, **kwargs)
        self.invalidate_packs()
        return out

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self.invalidate_packs()
        return out

    # -- loss execution (VGGLoss) --
    def run_forward(self, inputs, train):
        pred, gt, normalize = inputs[0], inputs[1], self._normalize
        n, _, H, W = pred.shape
        L.require_gpu(pred)
        plan = self._pool.acquire((n, H, W, self.dtype, normalize, True, pred.device))
        plan.set_input("pred", pred)
        plan.set_input("gt", gt)
        plan.run_forward()
        self.last_plan = plan
        if self.sign_log is not None:
            self.sign_log.append(plan.activation_signs())
        return plan, (plan.l1_out[:len(FEATURE_TAPS)].sum() / len(FEATURE_TAPS),)

    def run_backward(self, plan, inputs, grads, needs):
        pred = inputs[0]
        (go,) = grads
        gp = torch.empty(pred.shape, dtype=torch.float32, device=pred.device)
        plan.set_input_grad("pred", gp)
        plan.run_backward()
        return [gp * go, None]

    def perceptual_l1_into(self, pred, gt, normalize, out, value_scale, grad, grad_scale, accumulate):
        """Explicit-gradient form of perceptual_l1 (losses.LossTape): one plan forward over
        [pred | gt] writes value_scale * loss into out[0] (the five levels add into it);
        the plan backward, its seeds scaled by grad_scale, writes (accumulate=False) or adds
        grad_scale * d(loss)/d(pred) into grad (NCHW fp32).  No autograd node."""
        n, _, H, W = pred.shape
        L.require_gpu(pred)
        plan = self._pool.acquire((n, H, W, self.dtype, bool(normalize), True, pred.device))
        plan.busy = True
        try:
            plan.set_input("pred", pred)
            plan.set_input("gt", gt)
            plan.set_l1_loss(out, value_scale, grad_scale)
            plan.run_forward()
            if self.sign_log is not None:  # before a later loss call reuses the plan
                self.sign_log.append(plan.activation_signs())
            plan.set_input_grad("pred", grad, accumulate=accumulate)
            plan.run_backward()
        finally:
            plan.set_l1_loss(None)
            plan.busy = False
        self.last_plan = plan

    def perceptual_l1(self, pred, gt, normalize):
        self._normalize = bool(normalize)
        return PlanFunction.apply(self, 2, pred.float(), gt.float().detach())

    # -- plain feature extraction (reference signature) --
    def features_nhwc(self, img, normalize=False):
        n, _, H, W = img.shape
        plan = self._pool.acquire((n, H, W, self.dtype, bool(normalize), False, img.device))
        plan.set_input("pred", img.float())
        plan.run_forward()
        return [f.buf.t[..., f.c0:f.c0 + f.c] for f in plan.feats]

    def forward(self, img):
        with torch.no_grad():
            feats = self.features_nhwc(img)
        return tuple(f.permute(0, 3, 1, 2).float() for f in feats)
