"""ExtraTrainer on the MI355X path (reference runners/ExtraTrainer.py).

Extrapolation: frames 1, 2 (and their segmentations) -> frame 3 (and, with
`--num_pred_once k`, frames 3..2+k from one forward).  Same hot path as InterTrainer
(HRNet plan, RGBLoss + CE kernels, plan backward with in-backward RCCL buckets, fused
Adamax); the step body is the reference's l.234-323 factored into `step(data)`.

Loss keys follow the reference: `step_{i}_frame_{j}_coarse_{l1,gdl,vgg,ssim,ce}_loss`
and `loss_all` (l.286-315).

Reference defects this build does not reproduce:
  * l.65 `RGBLoss(args, sharp=False)` raises TypeError (RGBLoss has no `sharp`), so the
    reference train split cannot start; here RGBLoss(args) is constructed.
  * l.304-310 (rollout, `num_pred_step > 1`) reads the undefined `out_img` /
    `inpainted_img` / `out_seg`.  Here the rollout uses this step's prediction as the
    intended value: next input = [x[:, -3:], coarse_img] / [seg[:, -20:],
    onehot(argmax(coarse_seg))], gradients flowing back through coarse_img into the
    previous step (as the reference graph would, had it run).
  * l.188 `d[...]:0` (annotation, not assignment) only affects rank-0 logging.
With `--refine [--stage3]` (model ExtraRefineNet / ExtraStage3Net, build-defined two-stage
extrapolation nets for BASELINE config 5) the step adds the second-stage losses per scale
as the reference InterTrainer does (l.415-425).
The inpainting branch (`--inpaint`, InpaintUnet) has no model definition anywhere in the
reference tree and raises NotImplementedError here.
"""
from collections import OrderedDict

import torch

from .. import _lib as L
from ..data import batch_to
from ..losses import make_tape
from . import comm
from .InterTrainer import InterTrainer


def onehot_argmax(seg, n_classes=20):
    """torch.eye(20)[seg.argmax(1)].permute(0,3,1,2) (reference l.310), on device."""
    lab = seg.argmax(dim=1)
    return torch.nn.functional.one_hot(lab, n_classes).permute(0, 3, 1, 2).float().contiguous()


class ExtraTrainer(InterTrainer):
    def __init__(self, args):
        if getattr(args, "inpaint", False):
            raise NotImplementedError("--inpaint: InpaintUnet is not defined in the reference tree")
        args.syn_type = "extra"
        super().__init__(args)

    def get_input(self, data):
        """reference l.109-114"""
        x = torch.cat([data["frame1"], data["frame2"]], dim=1)
        seg = torch.cat([data["seg1"], data["seg2"]], dim=1) if self.args.mode == "xs2xs" else None
        vl = getattr(self.args, "vid_length", 1)
        gt_x = [data["frame" + str(i + 3)] for i in range(vl)]
        gt_seg = [data["seg" + str(i + 3)] if self.args.mode == "xs2xs" else None for i in range(vl)]
        return x, seg, gt_x, gt_seg

    def forward_backward(self, data):
        """Forward, losses and backward of one step (reference l.249-317); the gradient
        all-reduce and Adamax follow in InterTrainer.apply_gradients."""
        a = self.args
        npo, nps = getattr(a, "num_pred_once", 1), getattr(a, "num_pred_step", 1)
        if nps > 1:
            assert npo == 1, "rollout (num_pred_step > 1) requires num_pred_once == 1 (reference l.252-253)"
        assert not self.refine or nps == 1, "the two-stage nets train one-step predictions (num_pred_step 1)"
        data = batch_to(data, self.device)
        # a rollout runs HRNet's backward nps times into one flat gradient: reduce it once,
        # after the last backward (see GradSync.set_overlap)
        self.model.set_overlap(nps == 1 and not getattr(self, "no_overlap", False))
        xs2xs = a.mode == "xs2xs"
        tape = make_tape(self.device, self.W)
        last_rgb = torch.cat([data["frame1"], data["frame2"]], dim=1)
        last_seg = torch.cat([data["seg1"], data["seg2"]], dim=1) if xs2xs else None
        for ii in range(nps):
            g0 = 3 + ii * npo
            gt_x = torch.cat([data["frame" + str(i)] for i in range(g0, g0 + npo)], dim=1)
            gt_seg = torch.cat([data["seg" + str(i)] for i in range(g0, g0 + npo)], dim=1) if xs2xs else None
            x, seg = last_rgb, last_seg
            if getattr(a, "fix_init_frames", False):
                x = torch.cat([data["frame2"], x], dim=1)
                if xs2xs:
                    seg = torch.cat([data["seg2"], seg], dim=1)
            out = self.model(x, seg=seg, gt_x=gt_x, gt_seg=gt_seg)
            coarse_img, coarse_seg = out[0], out[1]
            for j in range(npo):
                prefix = "step_{}_frame_{}_coarse".format(ii + 1, j + 1)
                tape.rgb(self.RGBLoss, coarse_img[:, 3 * j:3 * j + 3], gt_x[:, 3 * j:3 * j + 3], False, prefix=prefix)
                if xs2xs:
                    tape.loss(prefix + "_ce_loss", L.LOSS_CE, coarse_seg[:, 20 * j:20 * j + 20],
                              gt_seg[:, 20 * j:20 * j + 20], a.ce_weight)
            if self.refine:
                self._refine_losses(tape, out, gt_x, "step_{}_frame_1_".format(ii + 1))
            if nps == 1:
                break
            last_rgb = torch.cat([x[:, -3:], coarse_img], dim=1)
            if xs2xs:
                last_seg = torch.cat([seg[:, -20:], onehot_argmax(coarse_seg)], dim=1)
        loss_dict = tape.loss_dict()
        for o in self._opts():
            o.zero_grad(set_to_none=True)
        tape.backward()  # reference `sync` divides loss_all by W in place (l.317, 760-765)
        return OrderedDict((k, v.detach()) for k, v in loss_dict.items())

    def _refine_losses(self, tape, out, gt_x, prefix):
        """Second-stage losses of the two-stage extrapolation nets (ExtraRefineNet /
        ExtraStage3Net), the structure of the reference InterTrainer's (l.415-425): per scale
        the refine RGBLoss and (--stage3) the stage-3 RGBLoss against the target frame
        resized to that scale; keys '<prefix>refine_<scale>_*' / '<prefix>stage3_<scale>_*'."""
        a = self.args
        for i in range(a.n_scales):
            tag = str(1 / (2 ** (a.n_scales - i - 1)))
            gts = self._scale_gt(gt_x, i)
            tape.rgb(self.refine_RGBLoss, out[2][i], gts, False, prefix=prefix + "refine_" + tag)
            if self.stage3:
                tape.rgb(self.refine_RGBLoss, out[3][i], gts, False, prefix=prefix + "stage3_" + tag)

    def validate(self):
        """Reference l.421-583: per (step, frame) L1 / PSNR / SSIM / IoU / VGG-cos."""
        a = self.args
        self.log.info("Validation epoch {} started".format(self.epoch))
        self.model.eval()
        npo, nps = getattr(a, "num_pred_once", 1), getattr(a, "num_pred_step", 1)
        crit = ["coarse_l1", "coarse_psnr", "coarse_ssim", "coarse_vgg", "coarse_iou"]
        from ..utils.net_utils import AverageMeter
        meters = OrderedDict()
        with torch.no_grad():
            for data in self.val_loader:
                data = batch_to(data, self.device)
                last_rgb = torch.cat([data["frame1"], data["frame2"]], dim=1)
                last_seg = torch.cat([data["seg1"], data["seg2"]], dim=1)
                d = OrderedDict()
                for i in range(nps):
                    g0 = 3 + i * npo
                    gt_x = torch.cat([data["frame" + str(k)] for k in range(g0, g0 + npo)], dim=1)
                    gt_seg = torch.cat([data["seg" + str(k)] for k in range(g0, g0 + npo)], dim=1)
                    x, seg = last_rgb, last_seg
                    if getattr(a, "fix_init_frames", False):
                        x = torch.cat([data["frame2"], x], dim=1)
                        seg = torch.cat([data["seg2"], seg], dim=1)
                    out = self.model(x, seg=seg, gt_x=gt_x, gt_seg=gt_seg)
                    coarse_img, coarse_seg = out[0], out[1]
                    for j in range(npo):
                        p = "step_{}_frame_{}_".format(i, j)
                        im = self.normalize(coarse_img[:, 3 * j:3 * j + 3])
                        gt = self.normalize(gt_x[:, 3 * j:3 * j + 3])
                        d[p + "coarse_l1"] = self.L1Loss(im, gt)
                        d[p + "coarse_psnr"] = self.PSNRLoss(im, gt)
                        d[p + "coarse_ssim"] = 1 - self.SSIMLoss(im, gt)
                        d[p + "coarse_iou"] = self.IoULoss.of_scores(coarse_seg[:, 20 * j:20 * j + 20],
                                                                     gt_seg[:, 20 * j:20 * j + 20])
                        d[p + "coarse_vgg"] = self.VGGCosLoss(im, gt, False)
                    if nps == 1:
                        break
                    last_rgb = torch.cat([x[:, -3:], coarse_img], dim=1)
                    last_seg = torch.cat([seg[:, -20:], onehot_argmax(coarse_seg)], dim=1)
                d = comm.sync_losses(d, self.W)
                if self.rank == 0:
                    for k, v in d.items():
                        meters.setdefault(k, AverageMeter()).update(float(v), data["frame1"].size(0) * self.W)
        res = OrderedDict((k, m.avg) for k, m in meters.items())
        if self.rank == 0:
            self.log.info("Epoch [{}] Evaluation: ".format(self.epoch) + " ".join(f"{k} [{v:.3f}]" for k, v in res.items()))
            self._scalars("val/score", res)
        return res

    def save_checkpoint(self):
        return super().save_checkpoint()


__all__ = ["ExtraTrainer", "onehot_argmax", "L"]
