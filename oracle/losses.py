"""Oracle: losses / metrics of the hot path, CPU fp32 restatements.

Reference: losses.py:18-48 (gaussian, create_window, _ssim), 63-87 (SSIM),
103-116 (PSNR), 122-131 (IoU), 137-151 (GDLLoss), 157-180 (VGGLoss),
182-207 (VGGCosineLoss), 213-241 (RGBLoss), 247-256 (GANScalarLoss);
utils/net_utils.py:11-23 (preprocess_norm); nets/vgg.py:11-54 (my_vgg);
runners/InterTrainer.py:414 (30 * CrossEntropy(seg, argmax(gt_seg))).
"""
from collections import OrderedDict
from math import exp

import torch
import torch.nn.functional as F

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def synthetic_vgg19_state(seed=19):
    """Deterministic stand-in for torchvision's pretrained VGG19 (no network access):
    kaiming-normal (fan_out, relu) weights from a private generator, zero biases."""
    gen = torch.Generator().manual_seed(seed)
    state, idx, cin = {}, 0, 3
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


def gaussian_window(window_size=11, sigma=1.5, dtype=torch.float32):
    """losses.py:18-26: the 1-D gaussian and its outer product are formed in the default dtype
    (torch.Tensor(list)) -- `dtype` here: that of the images, so a float64 run builds it in float64
    as the reference does under a float64 default -- then rounded to fp32 (`.float()`)"""
    g = torch.tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2)) for x in range(window_size)],
                     dtype=dtype)
    g = g / g.sum()
    return (g[:, None] @ g[None, :]).float()


def ssim_value(img1, img2, window_size=11):
    c = img1.shape[1]
    w = gaussian_window(window_size, dtype=img1.dtype).to(img1.dtype).expand(c, 1, window_size, window_size).contiguous()
    p = window_size // 2
    mu1 = F.conv2d(img1, w, padding=p, groups=c)
    mu2 = F.conv2d(img2, w, padding=p, groups=c)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, w, padding=p, groups=c) - mu1_sq
    s2 = F.conv2d(img2 * img2, w, padding=p, groups=c) - mu2_sq
    s12 = F.conv2d(img1 * img2, w, padding=p, groups=c) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return m.mean()


def ssim_loss(a, b):
    return 1 - ssim_value(a, b)


def l1_loss(a, b):
    return (a - b).abs().mean()


def gdl_loss(a, b):
    w = a.shape[-1]
    h = a.shape[-2]
    wa, ha = a[:, :, :, 1:] - a[:, :, :, :w - 1], a[:, :, 1:, :] - a[:, :, :h - 1, :]
    wb, hb = b[:, :, :, 1:] - b[:, :, :, :w - 1], b[:, :, 1:, :] - b[:, :, :h - 1, :]
    return ((wa - wb).abs().mean() + (ha - hb).abs().mean()) / 2


def psnr(pred, gt, max_level=1):
    out = 0
    for i in range(pred.shape[0]):
        d = torch.mean((pred[i] - gt[i]) ** 2)
        out += 10 * torch.log10(max_level * max_level / d)
    return out / pred.shape[0]


def preprocess_norm(x):
    mean = torch.tensor([0.485, 0.456, 0.406])[None, :, None, None]
    std = torch.tensor([0.229, 0.224, 0.225])[None, :, None, None]
    return (x - mean) / std


def _relu(x, masks, name):
    """ReLU; with `masks` (plan buffer name -> bool NCHW tensor) the branch is imposed, as
    hrnet._lrelu does for LeakyReLU (test support for fp64-vs-fp32 gradient checks)."""
    if masks is None or name not in masks:
        return F.relu(x)
    return torch.where(masks[name][:, :x.shape[1]].to(x.device), x, torch.zeros_like(x))


def vgg_features(state, img, masks=None):
    """my_vgg.forward: relu1_2, relu2_2, relu3_4, relu4_4, relu5_4 with AvgPool2d(2,2).
    masks: imposed ReLU branches keyed by the VGG plan's buffer names ('vgg<idx>')."""
    feats, x, idx = [], img, 0
    for v in VGG19_CFG:
        if v == "M":
            if idx == 36:
                break
            x = F.avg_pool2d(x, 2, 2)
            idx += 1
            continue
        x = _relu(F.conv2d(x, state[f"features.{idx}.weight"], state[f"features.{idx}.bias"], padding=1), masks,
                  f"vgg{idx}")
        idx += 2
        if idx in (4, 9, 18, 27, 36):
            feats.append(x)
    return feats


def _half(masks, lo, hi):
    return None if masks is None else {k: v[lo:hi] for k, v in masks.items()}


def vgg_loss(state, a, b, normed=True, masks=None):
    """masks: the VGG loss plan's ReLU branches over its [a | b] batch (2B images)."""
    if not normed:
        a, b = preprocess_norm(a).to(a.dtype), preprocess_norm(b).to(b.dtype)
    n = a.shape[0]
    fa, fb = vgg_features(state, a, _half(masks, 0, n)), vgg_features(state, b, _half(masks, n, 2 * n))
    return sum((x - y).abs().mean() for x, y in zip(fa, fb)) / len(fa)


def vgg_cosine(state, a, b, normed=True):
    if not normed:
        a, b = preprocess_norm(a), preprocess_norm(b)
    fa, fb = vgg_features(state, a), vgg_features(state, b)
    s = 0
    for x, y in zip(fa, fb):
        x = x / torch.sqrt(torch.sum(x ** 2, dim=1, keepdim=True))
        y = y / torch.sqrt(torch.sum(y ** 2, dim=1, keepdim=True))
        s += torch.mean(torch.sum(x * y, dim=1))
    return s / len(fa)


def seg_ce(logits, onehot):
    return F.cross_entropy(logits, torch.argmax(onehot, dim=1))


def rgb_loss(state, pred, gt, normed, w=(80.0, 80.0, 20.0, 20.0), prefix="coarse", vmasks=None):
    """RGBLoss.forward (losses.py:223-241) with the default weights (options.py:122-141).
    vmasks: imposed VGG ReLU branches (see vgg_loss)."""
    return OrderedDict([
        (f"{prefix}_l1_loss", w[0] * l1_loss(pred, gt)),
        (f"{prefix}_gdl_loss", w[1] * gdl_loss(pred, gt)),
        (f"{prefix}_vgg_loss", w[2] * vgg_loss(state, pred, gt, normed, vmasks)),
        (f"{prefix}_ssim_loss", w[3] * ssim_loss(pred, gt)),
    ])


def gan_hinge(x, is_target_true=True, weight=1.0):
    return weight * (F.relu(1 - x).mean() if is_target_true else F.relu(x + 1).mean())
