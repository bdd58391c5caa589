"""Reference utils/net_utils.py helpers on the MI355X path.

FlowWrapper (l.89-114) / warp (l.116-121) / warp_back (l.124-129): bilinear flow warp with
zero padding and align_corners=True (torch 1.0.1 grid_sample semantics) as one HIP kernel
per direction (dvie_warp_fwd / dvie_warp_bwd); preprocess_norm (l.11-23),
transform_seg_one_hot (l.33-50), AverageMeter (l.72-87).
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib as L


class _WarpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, flow, align_corners):
        L.require_gpu(x)
        x = x.float().contiguous()
        flow = flow.float().contiguous()
        n, c, h, w = x.shape
        assert flow.shape == (n, 2, h, w), (tuple(flow.shape), (n, 2, h, w))
        out = torch.empty_like(x)
        d = L.WarpDesc()
        d.img, d.flow, d.out = x.data_ptr(), flow.data_ptr(), out.data_ptr()
        d.n, d.c, d.h, d.w, d.align_corners = n, c, h, w, int(align_corners)
        L.check(L.load().dvie_warp_fwd(ctypes.byref(d), L.stream_ptr(x.device)), "warp fwd")
        ctx.save_for_backward(x, flow)
        ctx.ac = align_corners
        return out

    @staticmethod
    def backward(ctx, go):
        x, flow = ctx.saved_tensors
        go = go.float().contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None  # overwritten
        dflow = torch.empty_like(flow) if ctx.needs_input_grad[1] else None
        n, c, h, w = x.shape
        d = L.WarpDesc()
        d.img, d.flow, d.dout = x.data_ptr(), flow.data_ptr(), go.data_ptr()
        d.dimg = dx.data_ptr() if dx is not None else None
        d.dflow = dflow.data_ptr() if dflow is not None else None
        d.n, d.c, d.h, d.w, d.align_corners = n, c, h, w, int(ctx.ac)
        lib = L.load()
        nws = lib.dvie_warp_ws_floats(ctypes.byref(d))
        ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x.device)
        d.ws = ws.data_ptr()
        L.check(lib.dvie_warp_bwd(ctypes.byref(d), L.stream_ptr(x.device)), "warp bwd")
        return dx, dflow, None


def flow_warp(x, flow, align_corners=True):
    return _WarpFn.apply(x, flow, align_corners)


class FlowWrapper(nn.Module):
    """out = grid_sample(x, base_grid - flow), flow (N, 2, H, W) in normalized units."""

    def forward(self, x, flow):
        return flow_warp(x, flow, True)


def warp(frame, flow, opt, flowwarpper, mask):
    """Use mask before warping (reference l.116-121)."""
    out = [flowwarpper(frame, flow[:, :, i, :, :] * mask[:, i:i + 1, ...]).unsqueeze(1) for i in range(opt.vid_length)]
    return torch.cat(out, 1)


def warp_back(frame, flowback, opt, flowwarpper, mask):
    prev = [flowwarpper(frame[:, ii], -flowback[:, :, ii] * mask[:, ii:ii + 1, ...]).unsqueeze(1)
            for ii in range(opt.vid_length)]
    return torch.cat(prev, 1)


def preprocess_norm(input_tensor, cuda=True):
    mean = torch.tensor([0.485, 0.456, 0.406], device=input_tensor.device)[None, :, None, None]
    std = torch.tensor([0.229, 0.224, 0.225], device=input_tensor.device)[None, :, None, None]
    return (input_tensor - mean) / std


def transform_seg_one_hot(seg, n_cls, cuda=False):
    if seg.dim() != 3:
        raise ValueError(f"shape wrong {tuple(seg.shape)}")
    return torch.nn.functional.one_hot(seg.long(), n_cls).permute(0, 3, 1, 2).contiguous().float()


class AverageMeter:
    def __init__(self):
        self.reset()

    def reset(self):
        self.val = self.avg = self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


# the Cityscapes 19-class palette + "none" (reference utils/data_utils.py:86-107)
CITYSCAPES_COLORS = [
    (128, 64, 128), (244, 35, 232), (70, 70, 70), (102, 102, 156), (190, 153, 153), (153, 153, 153),
    (250, 170, 30), (220, 220, 0), (107, 142, 35), (152, 251, 152), (70, 130, 180), (220, 20, 60),
    (255, 0, 0), (0, 0, 142), (0, 0, 70), (0, 60, 100), (0, 80, 100), (0, 0, 230), (119, 11, 32), (0, 0, 0),
]


def vis_seg_mask(seg, n_classes, seg_id=False):
    """(B, C, H, W) scores (or (B, 1, H, W) ids with seg_id) -> (B, 3, H, W) palette colours
    in [0, 1] (reference utils/net_utils.py:57-70)."""
    assert seg.dim() == 4
    ids = seg.squeeze(1).long() if seg_id else seg.argmax(1)
    pal = torch.tensor(CITYSCAPES_COLORS, dtype=torch.float32, device=seg.device)
    return pal[ids].permute(0, 3, 1, 2).contiguous() / 255


def save_image(t, path):
    """torchvision.utils.save_image of one image (reference's save calls): (C, H, W) or
    (H, W) values scaled by 255, +0.5, clamped to [0, 255], a 1-channel image repeated to
    RGB, written as PNG."""
    import numpy as np
    from PIL import Image
    t = t.detach().float().cpu()
    if t.dim() == 2:
        t = t.unsqueeze(0)
    if t.shape[0] == 1:
        t = t.repeat(3, 1, 1)
    arr = t.mul(255).add(0.5).clamp(0, 255).to(torch.uint8).permute(1, 2, 0).numpy()
    Image.fromarray(np.ascontiguousarray(arr)).save(path)
