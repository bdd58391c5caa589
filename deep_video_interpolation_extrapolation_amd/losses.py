"""Losses and metrics of the frame-synthesis path (reference losses.py), on libdvie kernels.

Every training loss computes its value and d(loss)/d(pred) in one fused kernel pass
(deterministic block partials + a one-block fold); the autograd backward only scales the
stored gradient by the incoming scalar.  Class names, constructor arguments and return
conventions follow the reference:
  SSIM (l.63-87, returns 1 - mean ssim), PSNR (l.103-116), IoU (l.122-131),
  GDLLoss (l.137-151), VGGLoss (l.157-180), VGGCosineLoss (l.182-207),
  RGBLoss (l.213-241), GANScalarLoss (l.247-256), KLDLoss (l.50-60),
  plus L1Loss (nn.L1Loss) and SegCrossEntropy (nn.CrossEntropyLoss on argmax(one-hot),
  runners/InterTrainer.py:75,414).
"""
import ctypes
from collections import OrderedDict

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L
from .nets.vgg import my_vgg, vgg19_features


def _desc(kind, a, b, weight=1.0):
    d = L.LossDesc()
    d.kind = kind
    d.a, d.b = a.data_ptr(), b.data_ptr()
    d.a_sn, d.a_sc, d.a_sh, d.a_sw = a.stride()
    d.b_sn, d.b_sc, d.b_sh, d.b_sw = b.stride()
    d.bsz, d.ch, d.h, d.w = a.shape
    d.weight = weight
    d.dtype = L.F32
    return d


def run_loss(kind, a, b, want_grad, weight=1.0):
    """-> (value tensor [1] or [B] for MSE, grad (NCHW contiguous fp32) or None)"""
    L.require_gpu(a)
    assert a.dim() == 4 and b.dim() == 4 and a.dtype == torch.float32 and b.dtype == torch.float32
    if kind != L.LOSS_CE:
        assert a.shape == b.shape, (a.shape, b.shape)
    lib = L.load()
    d = _desc(kind, a, b, weight)
    npart = lib.dvie_loss_partial_count(ctypes.byref(d))
    part = torch.empty(max(1, npart), dtype=torch.float64, device=a.device)
    out = torch.empty(a.shape[0] if kind == L.LOSS_MSE else 1, dtype=torch.float32, device=a.device)
    grad = None
    if want_grad and kind != L.LOSS_MSE:
        grad = torch.empty(a.shape, dtype=torch.float32, device=a.device)
        d.grad = grad.data_ptr()
    ws = None
    if kind == L.LOSS_SSIM and grad is not None:
        ws = torch.empty(lib.dvie_loss_ws_floats(ctypes.byref(d)), dtype=torch.float32, device=a.device)
        d.ws = ws.data_ptr()
    d.partial, d.out = part.data_ptr(), out.data_ptr()
    L.check(lib.dvie_loss(ctypes.byref(d), L.stream_ptr(a.device)), f"loss kind {kind}")
    return out, grad


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kind, a, b):
        out, grad = run_loss(kind, a, b, ctx.needs_input_grad[1])
        ctx.grad = grad
        return out[0]

    @staticmethod
    def backward(ctx, go):
        g = ctx.grad * go if ctx.grad is not None else None
        ctx.grad = None
        return None, g, None


def _f32(t):
    return t if t.dtype == torch.float32 else t.float()


def l1_loss(a, b):
    return _LossFn.apply(L.LOSS_L1, _f32(a), _f32(b).detach())


def gdl_loss(a, b):
    return _LossFn.apply(L.LOSS_GDL, _f32(a), _f32(b).detach())


def ssim_loss(a, b):
    """1 - SSIM (reference SSIM.forward, losses.py:71-87)."""
    return _LossFn.apply(L.LOSS_SSIM, _f32(a), _f32(b).detach())


def seg_cross_entropy(logits, onehot):
    return _LossFn.apply(L.LOSS_CE, _f32(logits), _f32(onehot).detach())


class L1Loss(nn.Module):
    def forward(self, input, gt):
        return l1_loss(input, gt)


class GDLLoss(nn.Module):
    def forward(self, input, gt):
        return gdl_loss(input, gt)


class SSIM(nn.Module):
    def __init__(self, window_size=11, size_average=True):
        super().__init__()
        if window_size != 11 or not size_average:
            raise NotImplementedError("dvie SSIM: window 11, size_average=True (the reference configuration)")
        self.window_size, self.size_average = window_size, size_average

    def forward(self, img1, img2):
        return ssim_loss(img1, img2)


class SegCrossEntropy(nn.Module):
    """CrossEntropyLoss(logits, argmax(onehot, 1)) with the argmax fused."""

    def forward(self, logits, onehot):
        return seg_cross_entropy(logits, onehot)


class PSNR(nn.Module):
    def __init__(self, max_level=1):
        super().__init__()
        self.max_level = max_level

    def forward(self, pred, gt):
        assert pred.size() == gt.size()
        with torch.no_grad():
            mse, _ = run_loss(L.LOSS_MSE, _f32(pred), _f32(gt), False)
            return (10 * torch.log10(self.max_level * self.max_level / mse)).mean()


def _metric(kind, a, b, ch, dtype=None, strides=None, weight=1.0):
    """One metric reduction (dvie_loss kinds COSNHWC / IOU / ARGMAX_IOU) -> 0-dim fp32."""
    L.require_gpu(a)
    lib = L.load()
    d = L.LossDesc()
    d.kind, d.a, d.b = kind, a.data_ptr(), b.data_ptr()
    sa, sb = strides if strides is not None else (a.stride(), b.stride())
    d.a_sn, d.a_sc, d.a_sh, d.a_sw = sa
    d.b_sn, d.b_sc, d.b_sh, d.b_sw = sb
    d.bsz, d.ch, d.h, d.w = a.shape[0], ch, a.shape[-2], a.shape[-1]
    d.weight = weight
    d.dtype = L.F32 if dtype is None else dtype
    part = torch.empty(max(1, lib.dvie_loss_partial_count(ctypes.byref(d))), dtype=torch.float64, device=a.device)
    out = torch.empty(1, dtype=torch.float32, device=a.device)
    d.partial, d.out = part.data_ptr(), out.data_ptr()
    L.check(lib.dvie_loss(ctypes.byref(d), L.stream_ptr(a.device)), f"metric kind {kind}")
    return out[0]


class IoU(nn.Module):
    """Reference losses.py:122-131: fraction of pixels whose labels agree (a pixel
    accuracy, named IoU there).  pred / gt: (B, H, W) integer label maps."""

    def forward(self, pred, gt):
        assert pred.size() == gt.size()
        assert pred.dim() == 3
        a, b = pred.long(), gt.long()
        return _metric(L.LOSS_IOU, a, b, 1,
                       strides=((a.stride(0), 0, a.stride(1), a.stride(2)), (b.stride(0), 0, b.stride(1), b.stride(2))))

    @staticmethod
    def of_scores(pred_scores, gt_scores):
        """IoU(argmax(pred_scores, 1), argmax(gt_scores, 1)) with both argmaxes fused into
        the reduction (validate, runners/InterTrainer.py:615-624)."""
        assert pred_scores.shape == gt_scores.shape and pred_scores.dim() == 4
        a, b = _f32(pred_scores), _f32(gt_scores)
        return _metric(L.LOSS_ARGMAX_IOU, a, b, a.shape[1])


class VGGLoss(nn.Module):
    """Reference losses.py:157-180: mean over 5 taps of L1(vgg(pred), vgg(gt))."""

    def __init__(self, weights=None):
        super().__init__()
        self.vgg_net = my_vgg(vgg19_features(weights))

    def forward(self, input, gt, normed=True):
        return self.vgg_net.perceptual_l1(input, gt, normalize=not normed)


class VGGCosineLoss(nn.Module):
    """Reference losses.py:182-207 (validation metric)."""

    def __init__(self, weights=None):
        super().__init__()
        self.vgg_net = my_vgg(vgg19_features(weights))

    def forward(self, input, gt, normed=True):
        """One VGG plan over [input | gt] (2B images), then per feature level one HIP
        reduction of the per-pixel channel cosine between the two halves (NHWC, in the
        plan's compute dtype); the mean over the 5 levels is the score."""
        assert input.shape == gt.shape
        n = input.shape[0]
        with torch.no_grad():
            feats = self.vgg_net.features_nhwc(torch.cat([_f32(input), _f32(gt)], 0), normalize=not normed)
            dt = L.BF16 if feats[0].dtype == torch.bfloat16 else L.F32
            scores = []
            for f in feats:
                a, b = f[:n], f[n:]
                sn, sh, sw, sc = a.stride()
                st = (sn, sc, sh, sw)
                scores.append(_metric(L.LOSS_COSNHWC, a.permute(0, 3, 1, 2), b.permute(0, 3, 1, 2), f.shape[-1],
                                      dtype=dt, strides=(st, st), weight=1.0 / len(feats)))
            return torch.stack(scores).sum()


class RGBLoss(nn.Module):
    """Reference losses.py:213-241: OrderedDict of weighted l1 / gdl / vgg / ssim."""

    def __init__(self, args, window_size=11, size_average=True, refine=False):
        super().__init__()
        self.refine = refine
        self.vgg_loss = VGGLoss()
        self.gdl_loss = GDLLoss()
        self.ssim_loss = SSIM(window_size, size_average)
        self.l1_loss = L1Loss()
        self.args = args

    def forward(self, input, gt, normed=True, prefix=""):
        l1 = self.l1_loss(input, gt)
        vgg = self.vgg_loss(input, gt, normed)
        ssim = self.ssim_loss(input, gt)
        gdl = self.gdl_loss(input, gt)
        a = self.args
        if not self.refine:
            w = (a.l1_weight, a.gdl_weight, a.vgg_weight, a.ssim_weight)
        else:
            w = (a.refine_l1_weight, a.refine_gdl_weight, a.refine_vgg_weight, a.refine_ssim_weight)
        return OrderedDict([
            (f"{prefix}_l1_loss", w[0] * l1),
            (f"{prefix}_gdl_loss", w[1] * gdl),
            (f"{prefix}_vgg_loss", w[2] * vgg),
            (f"{prefix}_ssim_loss", w[3] * ssim),
        ])


class GANScalarLoss(nn.Module):
    """Hinge GAN loss (reference losses.py:247-256)."""

    def __init__(self, weight):
        super().__init__()
        self.weight = weight

    def forward(self, input, is_target_True=True):
        if is_target_True:
            return self.weight * F.relu(1 - input).mean()
        return self.weight * F.relu(input + 1).mean()


class KLDLoss(nn.Module):
    """Reference losses.py:50-60."""

    def __init__(self, args):
        super().__init__()
        self.args = args

    def forward(self, mu, logvar):
        kld = -0.5 * torch.sum(1 + logvar - mu.pow(2) - logvar.exp())
        return kld / mu.size(0) * self.args.kld_weight
