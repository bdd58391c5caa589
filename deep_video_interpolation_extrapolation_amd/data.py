"""Clip datasets for the trainers (reference data.py:21-143, folder.py:76-312).

The Cityscapes PNG clips and PANet bbox pickles the reference reads from hard-coded
/data/linz paths are not available; `SyntheticClips` produces samples with exactly the
reference's sample-dict layout: frame{1..k} (3,H,W) fp32 in [-1,1], seg{1..k} (20,H,W)
fp32 one-hot, bboxes (3,4,5) zeros.  Sample i is seeded 1000+i so every
rank / run sees identical data.  The device-side Cityscapes clip pipeline is a "next"
row.
"""
import torch
from torch.utils.data import Dataset


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
