"""ExtraNet (reference nets/ExtraNet.py:8-17): extrapolation wrapper around HRNet; the
extrapolation two-stage nets ExtraRefineNet / ExtraStage3Net (build-defined, see there)."""
import torch.nn as nn

from .HRNet import HRNet as _HRNet
from .InterRefineNet import InterRefineNet, InterStage3Net


class ExtraNet(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        name = getattr(args, "coarse_model", "HRNet")
        if name != "HRNet":
            raise NotImplementedError(f"coarse_model {name}: only HRNet is on the MI355X path")
        self.coarse_model = _HRNet(args)

    def forward(self, input, seg=None, gt_x=None, gt_seg=None):
        cm = self.coarse_model
        if cm.fix_init or cm.inpaint_mask:
            import torch
            return cm(torch.cat([input, seg], dim=1))
        return cm.forward_split(input, seg)



def _one_frame(args):
    if getattr(args, "num_pred_once", 1) != 1 or getattr(args, "fix_init_frames", False) or \
            getattr(args, "inpaint_mask", False):
        raise NotImplementedError("the extrapolation two-stage nets predict one frame from two "
                                  "(num_pred_once 1, no fix_init_frames / inpaint_mask)")


class ExtraRefineNet(InterRefineNet):
    """Extrapolation two-stage net, defined by this build: BASELINE config 5 names a
    two-stage extrapolation model, and the reference has none that runs (RefineGAN /
    RefineNet read undefined options, nets/RefineGAN.py:14-45; its ExtraTrainer has no
    second stage).  It is the composition of nets/InterRefineNet.py:8-31 with the
    extrapolation HRNet (frames 1, 2 -> frame 3; with one predicted frame its shapes equal
    the interpolation HRNet's, nets/HRNet.py:351-356): coarse HRNet, then SRNRefine on
    [clamp(coarse), softmax(coarse seg), frames + seg_encoder(seg_k)], all detached.
    forward(input, seg, gt_x, gt_seg) keeps ExtraNet's signature."""

    def __init__(self, args):
        _one_frame(args)
        super().__init__(args)

    def forward(self, input, seg=None, gt_x=None, gt_seg=None):
        return InterRefineNet.forward(self, input, seg=seg, gt_seg=gt_seg)


class ExtraStage3Net(InterStage3Net):
    """ExtraRefineNet + the stage-3 MSResAttnRefine on the last refine output, the two
    input frames as its attention neighbours (nets/InterRefineNet.py:33-53 composition on
    extrapolation inputs)."""

    def __init__(self, args):
        _one_frame(args)
        super().__init__(args)

    def forward(self, input, seg=None, gt_x=None, gt_seg=None):
        return InterStage3Net.forward(self, input, seg=seg, gt_seg=gt_seg)
