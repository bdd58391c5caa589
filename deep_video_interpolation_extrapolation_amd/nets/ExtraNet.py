"""ExtraNet (reference nets/ExtraNet.py:8-17): extrapolation wrapper around HRNet."""
import torch.nn as nn

from .HRNet import HRNet as _HRNet


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
