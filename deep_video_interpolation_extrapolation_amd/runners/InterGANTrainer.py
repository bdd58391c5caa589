"""InterGANTrainer on the MI355X path (reference runners/InterGANTrainer.py).

The step body (reference l.359-456) factored into `step(data)`:
  InterGANNet forward (HRNet plan, HIP softmax, D(fake.detach()), D(real), frozen-D(fake)
  discriminator plans)  ->  RGBLoss on [0,1] images (l.395) + 30*CE + hinge GAN losses
  (GANScalarLoss, l.409-422) [+ KLD with a VAE coarse model]  ->  one backward of the sum
  (generator, discriminator and softmax adjoints on HIP; RCCL buckets for the HRNet
  gradients inside the backward, one all-reduce per discriminator after it)  ->  fused
  Adamax (generator) and fused Adam (discriminators, l.110-112).
Loss keys and order follow the reference: coarse_{l1,gdl,vgg,ssim}_loss, coarse_ce_loss,
[coarse_kld_loss], coarse_frame_loss, disc_frame_real_loss, disc_frame_fake_loss,
coarse_video_loss, disc_video_real_loss, disc_video_fake_loss, loss_all.
"""
import os
from collections import OrderedDict

import torch

from .. import _lib as L
from ..data import batch_to
from ..losses import GANScalarLoss, KLDLoss, make_tape
from ..optim import Adam, Adamax
from . import comm
from .InterTrainer import InterTrainer

GAN_TRAIN_STEP = 0  # reference l.357: GAN terms are active from the first step


class InterGANTrainer(InterTrainer):
    def __init__(self, args):
        args.model = getattr(args, "model", "InterGANNet") or "InterGANNet"
        if args.model != "InterGANNet":
            args.model = "InterGANNet"
        # the discriminator optimizers must exist before a resume loads their state
        # (reference l.106-139: every optimizer is built, then load_checkpoint)
        self._defer_load = True
        super().__init__(args)
        a, m = self.args, self.model.module
        if not getattr(a, "train_coarse", False):
            m.set_net_grad(m.coarse_model, False)
        for kind in ("frame_disc", "video_disc"):
            if getattr(a, kind, False) and not getattr(a, "train_" + kind, False):
                m.set_net_grad(getattr(m, kind + "_model"), False)
        if a.split == "train":
            if getattr(a, "vae", False):
                self.KLDLoss = KLDLoss(a)
            if getattr(a, "frame_disc", False):
                self.FrameDisc_DLoss = GANScalarLoss(weight=a.frame_disc_disc_weight)
                self.FrameDisc_GLoss = GANScalarLoss(weight=a.frame_disc_gen_weight)
                self.frame_disc_opt = Adam(list(m.frame_disc_model.parameters()), lr=a.frame_disc_learning_rate)
            if getattr(a, "video_disc", False):
                self.VideoDisc_DLoss = GANScalarLoss(weight=a.video_disc_disc_weight)
                self.VideoDisc_GLoss = GANScalarLoss(weight=a.video_disc_gen_weight)
                self.video_disc_opt = Adam(list(m.video_disc_model.parameters()), lr=a.video_disc_learning_rate)
        if getattr(a, "resume", False) or (a.split != "train" and not getattr(a, "checkepoch_range", False)):
            self.load_checkpoint()  # reference l.138-139

    def get_input(self, data):
        """reference l.368-374 (interpolation: frames 1, 3 -> 2)"""
        gt_x = data["frame2"]
        gt_seg = data["seg2"]
        x = torch.cat([data["frame1"], data["frame3"]], dim=1)
        seg = torch.cat([data["seg1"], data["seg3"]], dim=1)
        return x, seg, gt_x, gt_seg

    def _predict(self, x, seg, gt_x, gt_seg):
        out = self.model(x, seg, gt_x, gt_seg)
        return out[0], out[1]

    def forward_backward(self, data):
        """InterGANNet forward, losses and one backward of their sum (reference
        l.359-442); apply_gradients runs the all-reduce and the optimizers."""
        a = self.args
        data = batch_to(data, self.device)
        x, seg, gt_x, gt_seg = self.get_input(data)
        bboxes = data.get("bboxes")
        out = self.model(x, seg, gt_x, gt_seg, bboxes=bboxes)
        (coarse_img, coarse_seg, mu, logvar, D_fake_frame, D_real_frame, D_fake_video, D_real_video,
         G_fake_frame, G_fake_video) = out[:10]
        self.global_step += 1
        on = 1.0 if self.global_step > GAN_TRAIN_STEP else 0.0
        prefix = "coarse"
        tape = make_tape(self.device, self.W)
        tape.rgb(self.RGBLoss, self.normalize(coarse_img), self.normalize(gt_x), False, prefix=prefix)
        tape.loss(prefix + "_ce_loss", L.LOSS_CE, coarse_seg, gt_seg, a.ce_weight)
        if getattr(a, "vae", False) and mu is not None:
            tape.scalar(prefix + "_kld_loss", self.KLDLoss(mu, logvar))
        if getattr(a, "frame_disc", False):
            tape.scalar("coarse_frame_loss", self.FrameDisc_GLoss(G_fake_frame, True) * on)
            tape.scalar("disc_frame_real_loss", self.FrameDisc_DLoss(D_real_frame, True) * on)
            tape.scalar("disc_frame_fake_loss", self.FrameDisc_DLoss(D_fake_frame, False) * on)
        if getattr(a, "video_disc", False):
            tape.scalar("coarse_video_loss", self.VideoDisc_GLoss(G_fake_video, True) * on)
            tape.scalar("disc_video_real_loss", self.VideoDisc_DLoss(D_real_video, True) * on)
            tape.scalar("disc_video_fake_loss", self.VideoDisc_DLoss(D_fake_video, False) * on)
        loss_dict = tape.loss_dict()
        for o in self._gan_opts().values():
            o.zero_grad(set_to_none=True)
        tape.backward()  # reference `sync` divides loss_all by W in place (l.442, 902-907)
        return OrderedDict((k, v.detach()) for k, v in loss_dict.items())

    def apply_gradients(self, reduce=True):
        a = self.args
        if reduce:
            self.model.finish()
        else:
            self.model.scale()
        opts = self._gan_opts()
        if getattr(a, "train_coarse", False):
            self.coarse_opt.step()
        for kind in ("frame_disc", "video_disc"):
            if getattr(a, kind, False) and getattr(a, "train_" + kind, False) and self.global_step > GAN_TRAIN_STEP:
                opts[kind].step()

    def _opts(self):
        return list(self._gan_opts().values())

    def _gan_opts(self):
        o = OrderedDict(coarse=self.coarse_opt)
        if hasattr(self, "frame_disc_opt"):
            o["frame_disc"] = self.frame_disc_opt
        if hasattr(self, "video_disc_opt"):
            o["video_disc"] = self.video_disc_opt
        return o

    # ---------------- checkpoints (reference l.910-1000) ----------------
    def save_checkpoint(self):
        name = self._ckpt_name(self.args.model, self.args.session, self.epoch, getattr(self, "step_idx", 0),
                               self.args.path)
        os.makedirs(os.path.dirname(name), exist_ok=True)
        m = self.model.module
        d = {"session": self.args.session, "epoch": self.epoch + 1,
             "coarse_model": m.coarse_model.state_dict(), "coarse_opt": self.coarse_opt.state_dict()}
        for kind in ("frame_disc", "video_disc"):
            if getattr(self.args, kind, False):
                d[kind + "_model"] = getattr(m, kind + "_model").state_dict()
                if hasattr(self, kind + "_opt"):
                    d[kind + "_opt"] = getattr(self, kind + "_opt").state_dict()
        torch.save(d, name)
        self.log.info("save model: {}".format(name))
        return name

    def load_checkpoint(self):
        """reference l.940-1059: weights gated by load_coarse / load_frame_disc /
        load_video_disc, optimizer states by train_* and load_* (train split), then the
        epoch bookkeeping of a resume / an evaluation split."""
        a = self.args
        name = self._ckpt_name(a.load_model, a.checksession, a.checkepoch, a.checkpoint, a.load_dir or ".")
        self.log.info("Loading checkpoint %s" % name)
        ckpt = torch.load(name, map_location="cpu", weights_only=True)
        m = self.model.module

        def merge(module, sd):
            cur = module.state_dict()
            cur.update(sd)
            module.load_state_dict(cur)

        if getattr(a, "load_coarse", False):
            merge(m.coarse_model, ckpt["coarse_model"])
        for kind in ("frame_disc", "video_disc"):
            if getattr(a, "load_" + kind, False):
                assert getattr(a, kind, False), "load_%s needs --%s" % (kind, kind)
                merge(getattr(m, kind + "_model"), ckpt[kind + "_model"])
        if a.split == "train":
            if getattr(a, "train_coarse", False) and getattr(a, "load_coarse", False):
                self.coarse_opt.load_state_dict(ckpt["coarse_opt"])
            for kind in ("frame_disc", "video_disc"):
                if getattr(a, "train_" + kind, False) and getattr(a, "load_" + kind, False):
                    assert getattr(a, kind, False)
                    getattr(self, kind + "_opt").load_state_dict(ckpt[kind + "_opt"])
        if getattr(a, "resume", False):
            assert ckpt["epoch"] - 1 == a.checkepoch, [ckpt["epoch"], a.checkepoch]
            self.epoch = ckpt["epoch"]
        elif a.split != "train":
            assert ckpt["epoch"] - 1 == a.checkepoch, [ckpt["epoch"], a.checkepoch]
            self.epoch = ckpt["epoch"] - 1
        self.log.info("checkpoint loaded")
