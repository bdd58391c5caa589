"""InterNet (reference nets/InterNet.py:8-17): coarse_model(cat([frames, segs])) -> (rgb, seg).

The concat of the reference is not materialised: the two halves go to the HRNet plan as
separate NCHW inputs (HRNet.forward_split), which packs them straight into its NHWC stem
buffer.
"""
import torch.nn as nn

from .HRNet import HRNet as _HRNet


class InterNet(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        name = getattr(args, "coarse_model", "HRNet")
        if name != "HRNet":
            raise NotImplementedError(f"coarse_model {name}: only HRNet is on the MI355X path")
        self.coarse_model = _HRNet(args)

    def forward(self, input, seg=None):
        return self.coarse_model.forward_split(input, seg)
