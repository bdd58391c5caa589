"""Two-stage interpolation nets (reference nets/InterRefineNet.py:8-53).

InterRefineNet: the coarse HRNet, then the refinement net (SRNRefine) on
  [clamp(coarse_rgb, -1, 1), softmax(coarse_seg), frames + seg_encoder(seg_k)], all detached
  (the refine loss does not reach the coarse net); refine outputs clamped to [-10, 10].
InterStage3Net: additionally the stage-3 net (MSResAttnRefine) on the last refine output
  (clamped to [-1, 1], detached), softmax(coarse_seg) and the input frames / segs; its
  outputs clamped to [-10, 10], plus its flow maps.

The seg encoder features are not recomputed: the HRNet plan already evaluates
seg_encoder(seg_k) for its stem and exports the stem concat [frames, enc(seg_0),
enc(seg_1)] as a detached side output (`export_stem`), which is exactly the reference's
encoded_feat.  softmax(coarse_seg) runs on the HIP channel-softmax kernel.
"""
import torch.nn as nn

from .HRNet import HRNet
from .InterGANNet import channel_softmax
from .refine import MSResAttnRefine, SRNRefine

_REFINE = {"SRNRefine": SRNRefine}
_STAGE3 = {"MSResAttnRefine": MSResAttnRefine}


def _coarse(args):
    name = getattr(args, "coarse_model", "HRNet")
    if name != "HRNet":
        raise NotImplementedError(f"coarse_model {name}: the two-stage nets take the HRNet coarse model")
    m = HRNet(args)
    m.export_stem = True
    return m


def _pick(table, name, what):
    if name not in table:
        # the reference's default refine_model 'refineUnet' names no class in its nets/
        # package (nets.__dict__['refineUnet'] raises there too)
        raise KeyError(f"{what} {name!r}: available {sorted(table)}")
    return table[name]


class InterRefineNet(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        self.coarse_model = _coarse(args)
        self.refine_model = _pick(_REFINE, getattr(args, "refine_model", "SRNRefine"), "refine_model")(args)

    def _coarse_pass(self, input, seg, gt_seg):
        coarse_rgb, coarse_seg = self.coarse_model.forward_split(input, seg)
        soft = channel_softmax(coarse_seg).detach()
        if getattr(self.args, "split", "train") == "val" and getattr(self.args, "with_gt_seg", False):
            soft = gt_seg
        enc = self.coarse_model.last_stem  # [frames, enc(seg_0), enc(seg_1)], detached
        return coarse_rgb, coarse_seg, soft, enc

    def forward(self, input, seg=None, gt_seg=None):
        coarse_rgb, coarse_seg, soft, enc = self._coarse_pass(input, seg, gt_seg)
        refine_rgbs = self.refine_model(coarse_rgb.detach().clamp(-1, 1), soft, enc)
        return coarse_rgb, coarse_seg, [img.clamp(-10, 10) for img in refine_rgbs]


class InterStage3Net(InterRefineNet):
    def __init__(self, args):
        super().__init__(args)
        self.stage3_model = _pick(_STAGE3, getattr(args, "stage3_model", "MSResAttnRefine"), "stage3_model")(args)

    def forward(self, input, seg=None, gt_seg=None):
        coarse_rgb, coarse_seg, soft, enc = self._coarse_pass(input, seg, gt_seg)
        refine_rgbs = self.refine_model(coarse_rgb.detach().clamp(-1, 1), soft, enc)
        refine_rgbs = [img.clamp(-1, 1) for img in refine_rgbs]
        re_refine, flow_maps = self.stage3_model(refine_rgbs[-1].detach(), soft, input, seg)
        return coarse_rgb, coarse_seg, refine_rgbs, [img.clamp(-10, 10) for img in re_refine], flow_maps
