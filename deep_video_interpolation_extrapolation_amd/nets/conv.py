"""HIP Conv2d: nn.Conv2d with the forward/backward on libdvie's implicit-GEMM kernels.

The reference's nets/conv.py is a non-importable copy of torch's conv module (its
relative imports, l.5-9, fail); this is where the build's convolution module lives.
`Conv2d` keeps nn.Conv2d's constructor, parameters (OIHW `weight`, `bias`), default
initialisation and state_dict keys.  Called on its own it lowers to a one-op engine
plan (NCHW->NHWC pack, conv with fused bias, NHWC->NCHW output); inside HRNet/VGG the
modules are only parameter holders and the whole network runs as one plan.
"""
import torch
import torch.nn as nn

from .. import _lib as L
from .. import engine as E
from ..runtime import PlanFunction, PlanPool, precision_of


class Conv2d(nn.Conv2d):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._dvie_pool = PlanPool(self._build_plan)

    def _build_plan(self, key):
        n, H, W, dtype, train, dev = key
        g = E.Graph(dtype)
        cin_p = E.rup(self.in_channels, 8)
        xb = g.buffer("x", H, W, cin_p)
        g.input_nchw(E.R(xb), "x", ext_c=self.in_channels, requires_grad=train)
        oh = (H + 2 * self.padding[0] - self.kernel_size[0]) // self.stride[0] + 1
        ow = (W + 2 * self.padding[1] - self.kernel_size[1]) // self.stride[1] + 1
        yb = g.buffer("y", oh, ow, E.rup(self.out_channels, 8), dtype=torch.float32, external=True)
        g.conv(E.R(xb), self, E.R(yb), name="conv")
        g.output("y", E.R(yb), self.out_channels)
        return g.compile(n, dev, backward=train)

    def run_forward(self, inputs, train):
        (x,) = inputs
        L.require_gpu(x)
        n, _, H, W = x.shape
        plan = self._dvie_pool.acquire((n, H, W, precision_of(), bool(train), x.device))
        plan.set_input("x", x)
        yb = plan.g.buffers[-1]
        y = torch.empty((n, yb.H, yb.W, yb.C), dtype=torch.float32, device=x.device)
        plan.set_output("y", y)
        plan.run_forward()
        return plan, (y.permute(0, 3, 1, 2)[:, :self.out_channels],)

    def run_backward(self, plan, inputs, grads, needs):
        (x,) = inputs
        (gy,) = grads
        for p in self.parameters():
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        plan.set_param_grads(accumulate=True)
        plan.set_output_grad("y", gy.float())
        gx = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        plan.set_input_grad("x", gx)
        plan.run_backward()
        return [gx]

    def forward(self, x):
        if self.padding_mode != "zeros" or self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("dvie Conv2d: zero padding, groups=1, dilation=1 only")
        if self.stride[0] != self.stride[1] or self.padding[0] != self.padding[1]:
            raise NotImplementedError("dvie Conv2d: square stride/padding only")
        params = [self.weight] + ([self.bias] if self.bias is not None else [])
        return PlanFunction.apply(self, 1, x.float(), *params)
