"""Clip datasets for the trainers (reference data.py:21-143, folder.py:76-312).

The Cityscapes PNG clips and PANet bbox pickles the reference reads from hard-coded
/data/linz paths are not available; `SyntheticClips` produces samples with exactly the
reference's sample-dict layout: frame{1..k} (3,H,W) fp32 in [-1,1], seg{1..k} (20,H,W)
fp32 one-hot, bboxes (3,4,5) zeros.  Sample i is seeded 1000+i so every
rank / run sees identical data.

`DeviceClips` is the device-side Cityscapes clip pipeline: the decoded
uint8 clips stay resident in HBM and one HIP launch (`dvie_clip_prep`) does the worker's
flip, pseudo-motion crop, to_tensor/normalize and 20-class one-hot for a whole batch.
"""
import ctypes
import random

import numpy as np
import torch
from torch.utils.data import Dataset

from . import _lib as L


class SyntheticClips(Dataset):
    def __init__(self, n, H, W, n_frames=3, n_classes=20):
        self.n, self.H, self.W, self.k, self.nc = n, H, W, n_frames, n_classes

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(1000 + i)
        out = {}
        for j in range(1, self.k + 1):
            out[f"frame{j}"] = torch.rand((3, self.H, self.W), generator=g) * 2 - 1
        for j in range(1, self.k + 1):
            lab = torch.randint(0, self.nc, (self.H, self.W), generator=g)
            out[f"seg{j}"] = torch.nn.functional.one_hot(lab, self.nc).permute(2, 0, 1).float()
        out["bboxes"] = torch.zeros((3, 4, 5))
        return out


def get_dataset(args):
    """-> (train_dataset, val_dataset).  Only synthetic clips are available offline."""
    n = getattr(args, "synthetic", 0) or 8
    k = 2 + max(1, getattr(args, "vid_length", 1)) if getattr(args, "syn_type", "inter") == "extra" else 3
    if getattr(args, "syn_type", "inter") == "extra" and getattr(args, "fix_init_frames", False):
        k += 1
    H, W = args.input_h, args.input_w
    return SyntheticClips(n, H, W, k), SyntheticClips(max(2, n // 4), H, W, k)


def batch_to(data, device):
    return {k: v.to(device, non_blocking=True) for k, v in data.items()}


def seq_crop_params(h0, w0, hc, wc, rng=np.random):
    """The reference's pseudo-motion crops (folder.py:125-149): three (h1, w1, hc, wc) for the
    forward / middle / backward frame, drawn with np.random in the reference's order.  The
    reference hard-codes 150 -> 128 on both axes; here (h0 - hc) and (w0 - wc)."""
    dh, dw = h0 - hc, w0 - wc
    if dh < 1 or dw < 1:
        raise ValueError(f"crop {hc}x{wc} needs a larger source frame than {h0}x{w0} (np.random.randint(0))")
    h_iv, w_iv = rng.randint(dh), rng.randint(dw)
    h_dir, w_dir = rng.randint(2), rng.randint(2)
    mid_h = rng.randint(h_iv // 2, dh - h_iv // 2)
    mid_w = rng.randint(w_iv // 2, dw - w_iv // 2)
    fh, bh = (mid_h - h_iv // 2, mid_h + h_iv // 2) if h_dir == 1 else (mid_h + h_iv // 2, mid_h - h_iv // 2)
    fw, bw = (mid_w - w_iv // 2, mid_w + w_iv // 2) if w_dir == 1 else (mid_w + w_iv // 2, mid_w - w_iv // 2)
    return (fh, fw, hc, wc), (mid_h, mid_w, hc, wc), (bh, bw, hc, wc)


class DeviceClips:
    """HBM-resident uint8 clip store with device-side preparation (reference DatasetFolder
    __getitem__, folder.py:197-261, for the frames / segs it returns).

    imgs: uint8 (N, T, H0, W0, 3) RGB as decoded; segs: uint8 (N, T, H0, W0) class ids or
    None.  split 'train': per clip a flip draw (random.randint(0, 2), folder.py:211) then the
    pseudo-motion crops to `crop` (T must be 3, as the reference indexes three crops);
    split 'val': whole frames, no flip.  `batch(indices)` returns the reference's collated
    dict: frame{1..T} (B,3,h,w) and seg{1..T} (B,20,h,w) fp32 on the device, bboxes zeros
    (B,3,4,5) (the detection bboxes are out of scope).  A label >= n_classes raises
    IndexError, as np.eye(20)[seg] does (strict=True: one device sync per batch)."""

    def __init__(self, imgs, segs=None, crop=None, split="train", n_classes=20, device=None, strict=True):
        device = torch.device(device) if device is not None else imgs.device
        if device.type != "cuda":
            raise L.DvieError("DeviceClips needs a GPU device (no CPU fallback)")
        if imgs.dtype != torch.uint8 or imgs.dim() != 5 or imgs.shape[-1] != 3:
            raise ValueError("imgs must be uint8 (N, T, H0, W0, 3)")
        self.imgs = imgs.to(device).contiguous()
        self.segs = segs.to(device).contiguous() if segs is not None else None
        if self.segs is not None and (self.segs.dtype != torch.uint8 or self.segs.shape != self.imgs.shape[:4]):
            raise ValueError("segs must be uint8 (N, T, H0, W0)")
        self.n, self.t, self.h0, self.w0 = self.imgs.shape[:4]
        self.split, self.nc, self.device, self.strict = split, n_classes, device, strict
        if split == "train":
            if crop is None or self.t != 3:
                raise ValueError("train split needs a crop size and 3-frame clips (folder.py:225-229)")
            self.hc, self.wc = crop
        else:
            self.hc, self.wc = self.h0, self.w0
        self._bad = torch.zeros(1, dtype=torch.int32, device=device)

    def __len__(self):
        return self.n

    def draw_params(self, batch, rng_np=np.random, rng_py=random):
        """(B, T, 3) int32 {flip, h1, w1}, drawn in the reference's per-sample order."""
        out = np.zeros((batch, self.t, 3), dtype=np.int32)
        if self.split != "train":
            return out
        for b in range(batch):
            flip = 1 if rng_py.randint(0, 2) else 0
            for i, (h1, w1, _, _) in enumerate(seq_crop_params(self.h0, self.w0, self.hc, self.wc, rng_np)):
                out[b, i] = (flip, h1, w1)
        return out

    def batch(self, indices, params=None):
        idx = torch.as_tensor(np.asarray(indices, dtype=np.int32)).to(self.device, non_blocking=True)
        B = int(idx.numel())
        if params is None:
            params = self.draw_params(B)
        params = np.ascontiguousarray(params, dtype=np.int32)
        if params.shape != (B, self.t, 3):
            raise ValueError(f"params must be (B, T, 3), got {params.shape}")
        if self.split == "train":
            h1, w1 = params[..., 1], params[..., 2]
            if (h1 < 0).any() or (w1 < 0).any() or (h1 + self.hc > self.h0).any() or (w1 + self.wc > self.w0).any():
                raise ValueError("crop outside the source frame")
        if (np.asarray(indices) < 0).any() or (np.asarray(indices) >= self.n).any():
            raise IndexError("clip index out of range")
        prm = torch.from_numpy(params).to(self.device, non_blocking=True)
        frames = torch.empty((self.t, B, 3, self.hc, self.wc), dtype=torch.float32, device=self.device)
        segs = (torch.empty((self.t, B, self.nc, self.hc, self.wc), dtype=torch.float32, device=self.device)
                if self.segs is not None else None)
        d = L.ClipDesc()
        d.img, d.idx, d.params, d.frames = self.imgs.data_ptr(), idx.data_ptr(), prm.data_ptr(), frames.data_ptr()
        if segs is not None:
            self._bad.zero_()
            d.seg, d.segs, d.bad = self.segs.data_ptr(), segs.data_ptr(), self._bad.data_ptr()
        d.b, d.t, d.h0, d.w0, d.hc, d.wc, d.n_classes = B, self.t, self.h0, self.w0, self.hc, self.wc, self.nc
        L.check(L.load().dvie_clip_prep(ctypes.byref(d), L.stream_ptr(self.device)), "clip prep")
        if segs is not None and self.strict and int(self._bad.item()):
            raise IndexError(f"segmentation label >= {self.nc} in the batch (np.eye({self.nc}) would raise)")
        out = {}
        for i in range(self.t):
            out[f"frame{i + 1}"] = frames[i]
            out[f"seg{i + 1}"] = segs[i] if segs is not None else torch.zeros((B, 1, 1), device=self.device)
        out["bboxes"] = torch.zeros((B, 3, 4, 5), device=self.device)
        return out

    def epoch(self, batch_size, rank=0, world=1, seed=0, drop_last=True):
        """Rank-strided shards of a seeded permutation (DistributedSampler semantics), one
        prepared batch per iteration."""
        perm = np.random.RandomState(seed).permutation(self.n)
        per = self.n // world if drop_last else -(-self.n // world)
        mine = perm[rank::world][:per]
        for s in range(0, len(mine) - (batch_size - 1 if drop_last else 0), batch_size):
            yield self.batch(mine[s:s + batch_size])


def load_clip_store(path, split, crop, device):
    """DeviceClips from a decoded uint8 store (npz, loaded without pickle).  Keys: imgs
    (N, 3, H0, W0, 3) and optional segs (N, 3, H0, W0) for training; val_imgs / val_segs
    for validation (fall back to imgs / segs).  The store is copied to HBM once."""
    with np.load(path, allow_pickle=False) as z:
        pre = "val_" if split != "train" and "val_imgs" in z.files else ""
        imgs = torch.from_numpy(np.ascontiguousarray(z[pre + "imgs"]))
        segs = torch.from_numpy(np.ascontiguousarray(z[pre + "segs"])) if pre + "segs" in z.files else None
    return DeviceClips(imgs, segs, crop=crop if split == "train" else None,
                       split="train" if split == "train" else "val", device=device)


class DeviceClipLoader:
    """DataLoader stand-in over `DeviceClips` (the reference's DataLoader + DistributedSampler
    pair, InterTrainer.py:86-96): each rank iterates its rank-strided shard of a permutation
    seeded by the epoch (`set_epoch`, as DistributedSampler.set_epoch), one prepared batch of
    `batch_size` clips per step, already on the device.  Training (shuffle=True) drops the
    last partial batch (every rank runs the same number of steps, so the gradient
    all-reduce stays matched).  Validation (shuffle=False) covers every clip exactly as the
    reference's val loader does (InterTrainer.py:97-100: DistributedSampler with its
    defaults -- seed-0 permutation, padded to a multiple of W by wrapping -- and
    drop_last=False), so metrics average over the same set."""

    def __init__(self, clips, batch_size, rank=0, world=1, shuffle=True, seed=0):
        self.clips, self.bs, self.rank, self.world = clips, max(1, batch_size), rank, world
        self.shuffle, self.seed, self.ep = shuffle, seed, 0
        self.sampler = self

    def set_epoch(self, epoch):
        self.ep = epoch

    def _val_indices(self):
        from torch.utils.data.distributed import DistributedSampler
        return list(DistributedSampler(range(len(self.clips)), num_replicas=self.world, rank=self.rank))

    def __len__(self):
        if self.shuffle:
            return (len(self.clips) // self.world) // self.bs
        return -(-len(self._val_indices()) // self.bs)

    def __iter__(self):
        if self.shuffle:
            return self.clips.epoch(self.bs, self.rank, self.world, seed=self.seed + self.ep)
        mine = np.asarray(self._val_indices(), dtype=np.int64)
        return (self.clips.batch(mine[s:s + self.bs]) for s in range(0, len(mine), self.bs))
