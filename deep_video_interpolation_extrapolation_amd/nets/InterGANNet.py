"""InterGANNet (reference nets/InterGANNet.py:8-127) on the MI355X path.

Same constructor flags, submodule names (coarse_model, frame_disc_model, video_disc_model)
and 19-tuple return of forward.  The three discriminator passes of the reference run as
three plan executions: D(fake.detach()) and D(real) train the discriminator (parameter
gradients, batch-statistics BatchNorm updating the running statistics, as in the
reference's train-mode calls), then D(fake) with the discriminator frozen
(`set_net_grad(False)`, l.78-81) sends gradients into the generator only.

coarse_model: the reference calls coarse_model(low_input, gt_x, gt_seg) and unpacks
(rgb, seg, mu, logvar), which only VAEHRNet provides, and VAEHRNet only runs at 128x128
(SURVEY §0.4).  Here HRNet is accepted too (mu = logvar = None, no KLD term), which is
what makes the 512x1024 InterGAN configuration (BASELINE configs[3]) runnable.
Detection discriminators and TrackGen need a pretrained ResNet101 and PANet bbox tracks
(out of scope) and raise NotImplementedError.
"""
import ctypes

import torch
import torch.nn as nn

from .. import _lib as L


class _SoftmaxFn(torch.autograd.Function):
    """F.softmax(x, dim=1) for fp32 NCHW (any strides) on the HIP kernel."""

    @staticmethod
    def forward(ctx, x):
        L.require_gpu(x)
        n, c, h, w = x.shape
        y = torch.empty((n, c, h, w), dtype=torch.float32, device=x.device)
        d = L.SoftmaxDesc()
        d.x, d.y = x.data_ptr(), y.data_ptr()
        d.sn, d.sc, d.sh, d.sw = x.stride()
        d.n, d.c, d.h, d.w = n, c, h, w
        L.check(L.load().dvie_softmax_fwd(ctypes.byref(d), L.stream_ptr(x.device)), "softmax")
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        gy = gy.float().contiguous()
        gx = torch.empty_like(y)
        d = L.SoftmaxDesc()
        d.y, d.gy, d.gx = y.data_ptr(), gy.data_ptr(), gx.data_ptr()
        d.n, d.c, d.h, d.w = y.shape
        L.check(L.load().dvie_softmax_bwd(ctypes.byref(d), L.stream_ptr(y.device)), "softmax backward")
        return gx


def channel_softmax(x):
    return _SoftmaxFn.apply(x.float())


class InterGANNet(nn.Module):
    def __init__(self, args):
        super().__init__()
        import sys
        factory = sys.modules[__package__].__dict__  # nets.__dict__[name](args), as the reference
        self.args = args
        for flag in ("frame_det_disc", "video_det_disc", "track_gen"):
            if getattr(args, flag, False):
                raise NotImplementedError(f"--{flag}: needs pretrained ResNet101 / PANet bbox tracks (out of scope)")
        self.coarse_model = factory[args.coarse_model](args)
        self.frame_disc = bool(getattr(args, "frame_disc", False))
        self.video_disc = bool(getattr(args, "video_disc", False))
        if self.frame_disc:
            self.frame_disc_model = factory[args.frame_disc_model](args)
        if self.video_disc:
            self.video_disc_model = factory[args.video_disc_model](args)

    @staticmethod
    def set_net_grad(net, flag=True):
        for p in net.parameters():
            p.requires_grad = flag

    def forward(self, input, seg=None, gt_x=None, gt_seg=None, bboxes=None):
        cm = self.coarse_model
        if hasattr(cm, "forward_vae"):
            coarse_rgb, coarse_seg, mu, var = cm.forward_vae(input, seg, gt_x, gt_seg)
        else:
            coarse_rgb, coarse_seg = cm.forward_split(input, seg)
            mu = var = None
        gen_bbox = None
        loc_diff_loss = torch.zeros(1, device=coarse_rgb.device)
        soft = channel_softmax(coarse_seg)
        if not self.training:
            return (coarse_rgb, coarse_seg, mu, var) + (0,) * 13 + (gen_bbox, loc_diff_loss)
        D_fake_frame = D_real_frame = D_fake_video = D_real_video = None
        G_fake_frame = G_fake_video = None
        if self.frame_disc:
            D_fake_frame = self.frame_disc_model(coarse_rgb.detach(), soft.detach(), bboxes=bboxes)
            D_real_frame = self.frame_disc_model(gt_x, gt_seg, bboxes=bboxes)
        if self.video_disc:
            D_fake_video = self.video_disc_model(coarse_rgb.detach(), soft.detach(), input, seg, bboxes=bboxes)
            D_real_video = self.video_disc_model(gt_x, gt_seg, input, seg, bboxes=bboxes)
        # G pass with the discriminator frozen, then set_net_grad(True) as in the reference
        # (l.78-81, 93-97): every parameter is trainable afterwards, SpectralNorm u / v included
        if self.frame_disc:
            self.set_net_grad(self.frame_disc_model, False)
            G_fake_frame = self.frame_disc_model(coarse_rgb, soft, bboxes=bboxes)
            self.set_net_grad(self.frame_disc_model, True)
        if self.video_disc:
            self.set_net_grad(self.video_disc_model, False)
            G_fake_video = self.video_disc_model(coarse_rgb, soft, input, seg, bboxes=bboxes)
            self.set_net_grad(self.video_disc_model, True)
        return (coarse_rgb, coarse_seg, mu, var,
                D_fake_frame, D_real_frame, D_fake_video, D_real_video, G_fake_frame, G_fake_video,
                None, None, None, None, None, None, None, gen_bbox, loc_diff_loss)
