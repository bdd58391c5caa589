"""GPU parity of the device clip pipeline (dvie_clip_prep through data.DeviceClips)
against the oracle's PIL / numpy / torch restatement of the reference worker
(folder.py:207-261).  Byte work with a division and a subtraction: bit-exact
(torch.equal), train (crop + flip, vector path) and val (whole frame, odd width: scalar
path), a label >= 20 raising IndexError as np.eye(20) does, and frames without segs."""
import random

import numpy as np
import pytest
import torch

from oracle import clip as OC

pytestmark = pytest.mark.gpu


def _store(n, t, h, w, seed, hi=20):
    rs = np.random.RandomState(seed)
    return (rs.randint(0, 256, (n, t, h, w, 3), dtype=np.uint8), rs.randint(0, hi, (n, t, h, w), dtype=np.uint8))


def test_train_batch_matches_oracle(dev):
    from deep_video_interpolation_extrapolation_amd.data import DeviceClips
    imgs, segs = _store(5, 3, 150, 150, 11)
    dc = DeviceClips(torch.from_numpy(imgs), torch.from_numpy(segs), crop=(128, 128), split="train", device=dev)
    idx = [3, 0, 3, 4]
    params = dc.draw_params(len(idx), np.random.RandomState(7), random.Random(7))
    assert params[..., 0].any() and not params[..., 0].all()  # both flip branches covered
    out = dc.batch(idx, params)
    torch.cuda.synchronize()
    for b, k in enumerate(idx):
        crops = [tuple(params[b, i, 1:]) + (128, 128) for i in range(3)]
        fr, oh = OC.prep_clip(list(imgs[k]), list(segs[k]), int(params[b, 0, 0]), crops)
        for i in range(3):
            assert torch.equal(out[f"frame{i + 1}"][b].cpu(), fr[i])
            assert torch.equal(out[f"seg{i + 1}"][b].cpu(), oh[i])
    assert out["bboxes"].shape == (4, 3, 4, 5)


def test_val_batch_odd_width(dev):
    from deep_video_interpolation_extrapolation_amd.data import DeviceClips
    imgs, segs = _store(3, 3, 33, 70, 5)
    dc = DeviceClips(torch.from_numpy(imgs), torch.from_numpy(segs), split="val", device=dev)
    out = dc.batch([2, 1])
    for b, k in enumerate([2, 1]):
        fr, oh = OC.prep_clip(list(imgs[k]), list(segs[k]), 0, None)
        for i in range(3):
            assert torch.equal(out[f"frame{i + 1}"][b].cpu(), fr[i])
            assert torch.equal(out[f"seg{i + 1}"][b].cpu(), oh[i])


def test_bad_label_raises(dev):
    from deep_video_interpolation_extrapolation_amd.data import DeviceClips
    imgs, segs = _store(2, 3, 40, 40, 9)
    segs[1, 2, 5, 7] = 20
    dc = DeviceClips(torch.from_numpy(imgs), torch.from_numpy(segs), crop=(32, 32), device=dev)
    dc.batch([0], np.zeros((1, 3, 3), dtype=np.int32))  # clip 0 is clean
    with pytest.raises(IndexError):
        dc.batch([1], np.zeros((1, 3, 3), dtype=np.int32))


def test_frames_only_and_epoch(dev):
    from deep_video_interpolation_extrapolation_amd.data import DeviceClips
    imgs, _ = _store(6, 3, 36, 44, 2)
    dc = DeviceClips(torch.from_numpy(imgs), None, crop=(32, 40), device=dev)
    batches = list(dc.epoch(2, rank=1, world=2, seed=3))
    assert len(batches) == 1 and batches[0]["frame1"].shape == (2, 3, 32, 40)
    assert float(batches[0]["frame2"].abs().max()) <= 1.0
