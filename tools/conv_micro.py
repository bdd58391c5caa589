"""Launch one conv plan (forward only, or forward+backward) repeatedly, for rocprofv3
counter collection on a single kernel shape.
    python tools/conv_micro.py cin cout k stride H W [batch] [prec] [iters] [bwd]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402
from deep_video_interpolation_extrapolation_amd import engine as E  # noqa: E402
from deep_video_interpolation_extrapolation_amd.nets.conv import Conv2d  # noqa: E402

cin, cout, k, s, H, W = map(int, sys.argv[1:7])
B = int(sys.argv[7]) if len(sys.argv) > 7 else 8
prec = sys.argv[8] if len(sys.argv) > 8 else "bf16"
iters = int(sys.argv[9]) if len(sys.argv) > 9 else 20
bwd = len(sys.argv) > 10 and sys.argv[10] == "bwd"
dt = torch.bfloat16 if prec == "bf16" else torch.float32
dev = torch.device("cuda:0")
m = Conv2d(cin, cout, k, s, k // 2, bias=False).to(dev)
g = E.Graph(dt)
xb = g.buffer("x", H, W, E.rup(cin, 8))
oh, ow = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
yb = g.buffer("y", oh, ow, E.rup(cout, 8))
g.input_nchw(E.R(xb), "in", ext_c=cin, requires_grad=bwd)
g.conv(E.R(xb), m, E.R(yb), act=L.ACT_LRELU, name="conv")
m2 = Conv2d(E.rup(cout, 8), 8, 1, 1, 0, bias=False).to(dev)
zb = g.buffer("z", oh, ow, 8, dtype=torch.float32, external=True)
g.conv(E.R(yb), m2, E.R(zb), name="post")
g.output("z", E.R(zb), 8)
plan = g.compile(B, dev, backward=bwd)
inp = torch.randn(B, cin, H, W, device=dev)
plan.set_input("in", inp)
z = torch.empty(B, oh, ow, 8, device=dev)
plan.set_output("z", z)
if bwd:
    plan.set_output_grad("z", torch.randn(B, 8, oh, ow, device=dev))
    plan.set_input_grad("in", torch.empty_like(inp))
    for p in (m, m2):
        p.weight.grad = torch.zeros_like(p.weight)
    plan.set_param_grads(True)
for _ in range(iters):
    plan.run_forward()
    if bwd:
        plan.run_backward()
torch.cuda.synchronize()
print("done")
