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
    d.out_scale = 1.0
    d.dtype = L.F32
    return d


def run_loss(kind, a, b, want_grad, weight=1.0, out=None, out_scale=1.0, grad=None, beta=0):
    """-> (value tensor [1] or [B] for MSE, grad (NCHW contiguous fp32) or None).
    out / grad: caller-owned buffers (LossTape): out[0] receives out_scale * loss, grad
    receives (beta 0) or gains (beta 1) weight * d(loss)/d(a)."""
    L.require_gpu(a)
    assert a.dim() == 4 and b.dim() == 4 and a.dtype == torch.float32 and b.dtype == torch.float32
    if kind != L.LOSS_CE:
        assert a.shape == b.shape, (a.shape, b.shape)
    lib = L.load()
    d = _desc(kind, a, b, weight)
    d.out_scale = out_scale
    npart = lib.dvie_loss_partial_count(ctypes.byref(d))
    part = torch.empty(max(1, npart), dtype=torch.float64, device=a.device)
    if out is None:
        out = torch.empty(a.shape[0] if kind == L.LOSS_MSE else 1, dtype=torch.float32, device=a.device)
    else:
        assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() >= 1
    if grad is not None:
        assert kind != L.LOSS_MSE and grad.dtype == torch.float32 and grad.is_contiguous() and grad.shape == a.shape
        d.grad, d.beta = grad.data_ptr(), int(beta)
    elif want_grad and kind != L.LOSS_MSE:
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
    d.out_scale = 1.0
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


class LossTape:
    """Explicit-gradient assembly of one training step's loss: the trainers' loss_dict,
    loss_all = sum of its terms, and (loss_all / W).backward() (reference
    runners/InterTrainer.py:401-431, ExtraTrainer.py:302-317, InterGANTrainer.py:390-442).

    A native term (L1 / GDL / SSIM / CE kernel, VGG plan) writes weight * loss into its own
    slot of a step-local value vector (the kernel's out_scale) and adds
    (weight / W) * d(loss)/d(prediction) straight into that prediction's gradient buffer
    (the kernel's beta accumulation; VGG through its plan backward with scaled seeds).
    loss_all is one dvie_sum_f32 over the slots.  backward() then runs autograd from the
    predictions with those buffers as their gradients, plus any scalar term left to
    autograd (GAN hinge, KLD).  So the step issues no PyTorch kernel for loss weighting,
    summation, gradient scaling, gradient accumulation or the backward seed -- the same
    gradients as autograd through the per-term functions, summed in a fixed order."""

    CAP = 64

    def __init__(self, device, world=1):
        self.vals = torch.empty(self.CAP + 1, dtype=torch.float32, device=device)  # [terms | loss_all]
        self.n = 0
        self.items = []  # (key, slot index or a differentiable 0-dim tensor)
        self.inv_w = 1.0 / world
        self.sinks = {}  # id(prediction) -> [prediction, gradient buffer, written]
        self.device = device

    def _slot(self, key):
        if self.n >= self.CAP:
            raise RuntimeError("LossTape: more than %d native loss terms" % self.CAP)
        i = self.n
        self.n += 1
        self.items.append((key, i))
        return self.vals[i:i + 1]

    def _sink(self, t):
        e = self.sinks.get(id(t))
        if e is None:
            e = self.sinks[id(t)] = [t, torch.empty(t.shape, dtype=torch.float32, device=t.device), False]
        acc = e[2]
        e[2] = True
        return e[1], acc

    def loss(self, key, kind, pred, target, weight=1.0):
        """weight * loss(pred, target), loss one of L1 / GDL / SSIM / CE (target detached)."""
        pred, target = _f32(pred), _f32(target).detach()
        out = self._slot(key)
        g, acc = self._sink(pred) if pred.requires_grad else (None, 0)
        _run_into(kind, pred, target, out, weight, g, weight * self.inv_w, acc)

    def vgg(self, key, vgg_loss, pred, gt, normed=True, weight=1.0):
        """weight * VGGLoss(pred, gt) (losses.py:157-180 of the reference)."""
        pred, gt = _f32(pred), _f32(gt).detach()
        out = self._slot(key)
        if pred.requires_grad:
            g, acc = self._sink(pred)
            vgg_loss.vgg_net.perceptual_l1_into(pred, gt, not normed, out, weight, g, weight * self.inv_w, acc)
        else:
            with torch.no_grad():
                out.copy_(weight * vgg_loss(pred, gt, normed))

    def rgb(self, rgb_loss, input, gt, normed=True, prefix=""):
        """RGBLoss(input, gt, normed, prefix): its four weighted terms, same keys and order."""
        w = rgb_loss.weights()
        self.loss(f"{prefix}_l1_loss", L.LOSS_L1, input, gt, w[0])
        self.loss(f"{prefix}_gdl_loss", L.LOSS_GDL, input, gt, w[1])
        self.vgg(f"{prefix}_vgg_loss", rgb_loss.vgg_loss, input, gt, normed, w[2])
        self.loss(f"{prefix}_ssim_loss", L.LOSS_SSIM, input, gt, w[3])

    def scalar(self, key, v):
        """A differentiable 0-dim term left to autograd (GAN hinge, KLD)."""
        self.items.append((key, v))

    def loss_dict(self):
        """OrderedDict key -> 0-dim tensor (native slots are views of the value vector),
        'loss_all' last; loss_all carries autograd only through the scalar terms."""
        lib = L.load()
        tot = self.vals[self.CAP:self.CAP + 1]
        if self.n:
            L.check(lib.dvie_sum_f32(self.vals.data_ptr(), self.n, tot.data_ptr(), L.stream_ptr(self.device)),
                    "loss_all")
        else:
            tot.zero_()
        ld = OrderedDict()
        extra = None
        for key, v in self.items:
            if isinstance(v, int):
                ld[key] = self.vals[v]
            else:
                ld[key] = v
                extra = v if extra is None else extra + v
        self._extra = extra
        ld["loss_all"] = self.vals[self.CAP] if extra is None else self.vals[self.CAP] + extra
        return ld

    _seeds = {}

    def backward(self):
        """autograd from the predictions (their tape gradients) and the scalar terms."""
        tensors, grads = [], []
        for t, g, written in self.sinks.values():
            if written:
                tensors.append(t)
                grads.append(g)
        extra = getattr(self, "_extra", None)
        if extra is not None:
            key = (str(self.device), self.inv_w)
            seed = LossTape._seeds.get(key)
            if seed is None:  # created once per device and W, never inside a captured step
                seed = LossTape._seeds[key] = torch.full((), self.inv_w, dtype=torch.float32, device=self.device)
            tensors.append(extra)
            grads.append(seed.to(extra.dtype))
        if tensors:
            torch.autograd.backward(tensors, grads)
        self.sinks = {}


class AutogradTape:
    """LossTape's interface on the per-term autograd functions, as the reference writes the
    loss (`loss_dict[k] = w * loss_fn(...)`, loss_all = sum of torch.mean(v),
    (loss_all / W).backward()).  DVIE_LOSS_TAPE=0 selects it (A/B runs, cross-checks)."""

    def __init__(self, device, world=1):
        self.ld = OrderedDict()
        self.world = world

    def loss(self, key, kind, pred, target, weight=1.0):
        fn = {L.LOSS_L1: l1_loss, L.LOSS_GDL: gdl_loss, L.LOSS_SSIM: ssim_loss, L.LOSS_CE: seg_cross_entropy}[kind]
        self.ld[key] = weight * fn(pred, target)

    def rgb(self, rgb_loss, input, gt, normed=True, prefix=""):
        self.ld.update(rgb_loss(input, gt, normed, prefix=prefix))

    def scalar(self, key, v):
        self.ld[key] = v

    def loss_dict(self):
        loss = 0
        for v in self.ld.values():
            loss = loss + torch.mean(v)
        self.ld["loss_all"] = loss
        return self.ld

    def backward(self):
        (self.ld["loss_all"] / self.world).backward()


def make_tape(device, world=1):
    """The training step's loss assembly: LossTape, or AutogradTape under DVIE_LOSS_TAPE=0."""
    import os
    if os.environ.get("DVIE_LOSS_TAPE", "1") == "0":
        return AutogradTape(device, world)
    return LossTape(device, world)


def _run_into(kind, pred, target, out, weight, grad, gweight, acc):
    """one native loss term: out[0] = weight * loss, grad (+)= gweight * d(loss)/d(pred)."""
    lib = L.load()
    d = _desc(kind, pred, target, gweight)
    d.out_scale = weight
    npart = lib.dvie_loss_partial_count(ctypes.byref(d))
    part = torch.empty(max(1, npart), dtype=torch.float64, device=pred.device)
    if grad is not None:
        d.grad, d.beta = grad.data_ptr(), int(acc)
        if kind == L.LOSS_SSIM:
            ws = torch.empty(lib.dvie_loss_ws_floats(ctypes.byref(d)), dtype=torch.float32, device=pred.device)
            d.ws = ws.data_ptr()
    d.partial, d.out = part.data_ptr(), out.data_ptr()
    L.check(lib.dvie_loss(ctypes.byref(d), L.stream_ptr(pred.device)), f"loss kind {kind}")


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

    def weights(self):
        a = self.args
        if not self.refine:
            return (a.l1_weight, a.gdl_weight, a.vgg_weight, a.ssim_weight)
        return (a.refine_l1_weight, a.refine_gdl_weight, a.refine_vgg_weight, a.refine_ssim_weight)

    def forward(self, input, gt, normed=True, prefix=""):
        l1 = self.l1_loss(input, gt)
        vgg = self.vgg_loss(input, gt, normed)
        ssim = self.ssim_loss(input, gt)
        gdl = self.gdl_loss(input, gt)
        w = self.weights()
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
