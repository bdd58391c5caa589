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


def test_device_loader_shards_and_epochs(dev):
    """DeviceClipLoader: rank shards of one epoch partition the store, set_epoch reshuffles,
    and the unshuffled (val) order is the reference val sampler's (DistributedSampler defaults)."""
    from deep_video_interpolation_extrapolation_amd.data import DeviceClipLoader, DeviceClips
    imgs, segs = _store(8, 3, 20, 36, 5)
    dc = DeviceClips(torch.from_numpy(imgs), torch.from_numpy(segs), split="val", device=dev)
    key = lambda f: int(((f[0, 0, 0] * .5 + .5) * 255).round())  # first byte of a clip's frame 1
    firsts = {int(imgs[k, 0, 0, 0, 0]): k for k in range(8)}
    assert len(firsts) == 8
    seen = []
    for r in range(2):
        ld = DeviceClipLoader(dc, 2, rank=r, world=2, shuffle=True, seed=3)
        assert len(ld) == 2
        for b in ld:
            seen += [firsts[key(b["frame1"][i])] for i in range(b["frame1"].shape[0])]
    assert sorted(seen) == list(range(8))
    ld = DeviceClipLoader(dc, 2, rank=0, world=2, shuffle=True, seed=3)
    for ep in (0, 1):
        ld.set_epoch(ep)
        got = [firsts[key(b["frame1"][i])] for b in ld for i in range(2)]
        assert got == list(np.random.RandomState(3 + ep).permutation(8)[0::2])
    from torch.utils.data.distributed import DistributedSampler
    ld = DeviceClipLoader(dc, 2, rank=1, world=2, shuffle=False)
    want = list(DistributedSampler(range(8), num_replicas=2, rank=1))  # the reference val sampler
    assert [firsts[key(b["frame1"][i])] for b in ld for i in range(b["frame1"].shape[0])] == want


def test_main_launcher_clip_store(dev, tmp_path):
    """The launcher with --clip_store: one epoch of training on HBM-resident uint8 clips
    cropped on the GPU, the checkpoint, and validation on whole frames from the store."""
    from deep_video_interpolation_extrapolation_amd import main as M
    imgs, segs = _store(4, 3, 40, 72, 9)
    vimgs, vsegs = _store(2, 3, 32, 64, 10)
    store = tmp_path / "clips.npz"
    np.savez(store, imgs=imgs, segs=segs, val_imgs=vimgs, val_segs=vsegs)
    common = ["--syn_type", "inter", "--bs", "2", "--input_h", "32", "--input_w", "64", "--epochs", "1",
              "--save_dir", str(tmp_path / "log"), "--clip_store", str(store), "--nw", "0", "--precision", "fp32"]
    M.main(common + ["INTER", "--train_coarse"])
    run = next((tmp_path / "log").iterdir())
    ck = next((run / "checkpoint").iterdir())
    M.main(common + ["--split", "val", "--load_dir", str(run), "--checkepoch", "1", "--checkpoint",
                           ck.name.split("_")[-1][:-4], "--checksession", "0", "INTER", "--load_coarse"])
    assert "Epoch [1/1][1/2]" in (run / "experiment_train.log").read_text()
    assert "Evaluation" in (run / "experiment_val.log").read_text()
