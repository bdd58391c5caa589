"""Oracle (test infrastructure only): the reference DataLoader worker's clip preparation,
restated with the same library calls it makes.

* seq_crop_params: folder.py:125-149 get_seq_crop_params (np.random draws in the same
  order; the reference hard-codes 150 -> 128 on both axes, here (h0 - hc) and (w0 - wc),
  identical at the reference sizes).
* prep_clip: folder.py:207-247 (train) / 248-261 (val): PIL FLIP_LEFT_RIGHT on the full
  frame, torchvision F.crop(img, top=h1, left=w1, h, w) == PIL img.crop((w1, h1, w1+w, h1+h)),
  to_tensor (HWC uint8 -> CHW float / 255), normalize((.5,)*3, (.5,)*3), and
  np.eye(20)[seg] transposed to (20, h, w) float.
Parity: seq_crop_params and draw_flip are pinned to the reference itself (fixture G13,
tests/golden/clip_crops.npz, generated from folder.py:125-149, 166); prep_clip is pinned by
construction to those PIL / numpy / torch calls; the reference
DatasetFolder itself is not executed (its torchvision transforms are absent offline).
"""
import random

import numpy as np
import torch
from PIL import Image


def seq_crop_params(h0, w0, hc, wc, rng=np.random):
    """-> three (h1, w1, hc, wc) crops (forward, middle, backward frame) of a pseudo-motion."""
    dh, dw = h0 - hc, w0 - wc
    h_interval = rng.randint(dh)
    w_interval = rng.randint(dw)
    h_dir = rng.randint(2)
    w_dir = rng.randint(2)
    mid_h1 = rng.randint(h_interval // 2, dh - h_interval // 2)
    mid_w1 = rng.randint(w_interval // 2, dw - w_interval // 2)
    if h_dir == 1:
        for_h1, back_h1 = mid_h1 - h_interval // 2, mid_h1 + h_interval // 2
    else:
        for_h1, back_h1 = mid_h1 + h_interval // 2, mid_h1 - h_interval // 2
    if w_dir == 1:
        for_w1, back_w1 = mid_w1 - w_interval // 2, mid_w1 + w_interval // 2
    else:
        for_w1, back_w1 = mid_w1 + w_interval // 2, mid_w1 - w_interval // 2
    assert 0 <= for_h1 < dh and 0 <= mid_h1 < dh and 0 <= back_h1 < dh
    return (for_h1, for_w1, hc, wc), (mid_h1, mid_w1, hc, wc), (back_h1, back_w1, hc, wc)


def draw_flip(rng=random):
    """folder.py:211: isHorflip = randint(0, 2) (inclusive: flip with probability 2/3)."""
    return rng.randint(0, 2)


def prep_clip(imgs, segs, flip, crops, n_classes=20):
    """imgs: list of (H0, W0, 3) uint8; segs: list of (H0, W0) uint8 or None;
    crops: per-frame (h1, w1, hc, wc) or None (val: whole frame).
    -> (list of (3, h, w) fp32, list of (n_classes, h, w) fp32)"""
    frames, onehots = [], []
    for i, a in enumerate(imgs):
        im = Image.fromarray(a, "RGB")
        sg = Image.fromarray(segs[i], "L") if segs is not None else None
        if flip:
            im = im.transpose(Image.FLIP_LEFT_RIGHT)
            sg = sg.transpose(Image.FLIP_LEFT_RIGHT) if sg is not None else None
        if crops is not None:
            h1, w1, h, w = crops[i]
            im = im.crop((w1, h1, w1 + w, h1 + h))
            sg = sg.crop((w1, h1, w1 + w, h1 + h)) if sg is not None else None
        t = torch.from_numpy(np.array(im)).permute(2, 0, 1).contiguous().float().div(255)
        mean = torch.tensor([0.5, 0.5, 0.5]).view(3, 1, 1)
        frames.append(t.sub(mean).div(mean))
        if sg is not None:
            oh = np.eye(n_classes)[np.array(sg)]
            onehots.append(torch.from_numpy(np.transpose(oh, (2, 0, 1))).float())
    return frames, onehots
