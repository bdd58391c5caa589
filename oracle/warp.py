"""Oracle: bilinear flow warp, FlowWrapper (reference utils/net_utils.py:89-114),
warp / warp_back (l.116-129).  grid_sample with align_corners=True reproduces the pinned
torch 1.0.1 behaviour (fyp.yml:125)."""
import torch
import torch.nn.functional as F


def flow_warp(x, flow, align_corners=True):
    N, _, H, W = x.shape
    base = torch.zeros(N, H, W, 2)
    lin = torch.linspace(-1, 1, W) if W > 1 else torch.tensor([-1.0])
    base[:, :, :, 0] = torch.outer(torch.ones(H), lin).expand_as(base[:, :, :, 0])
    lin = torch.linspace(-1, 1, H) if H > 1 else torch.tensor([-1.0])
    base[:, :, :, 1] = torch.outer(lin, torch.ones(W)).expand_as(base[:, :, :, 1])
    grid = base - flow.transpose(1, 2).transpose(2, 3)
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=align_corners)


def warp(frame, flow, vid_length, mask):
    """flow (B, 2, T, H, W), mask (B, T, H, W) -> (B, T, C, H, W)"""
    return torch.cat([flow_warp(frame, flow[:, :, i] * mask[:, i:i + 1]).unsqueeze(1) for i in range(vid_length)], 1)


def warp_back(frame, flowback, vid_length, mask):
    return torch.cat([flow_warp(frame[:, i], -flowback[:, :, i] * mask[:, i:i + 1]).unsqueeze(1)
                      for i in range(vid_length)], 1)
