"""Diagnostic: gradient buffers (pre-activation gradients) of the HIP plan vs the fp64
oracle's autograd gradients of the same intermediates."""
import os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
os.environ["DVIE_PRECISION"] = sys.argv[1] if len(sys.argv) > 1 else "fp32"
import torch
import inputs
from oracle import hrnet as O
from deep_video_interpolation_extrapolation_amd import nets

dev = torch.device("cuda:0")
torch.manual_seed(1024)
m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet")).to(dev)
P0 = O.init_params(1024)
H, W = 32, 64
x, seg = inputs.hrnet_input(2, H, W)
g = torch.Generator().manual_seed(5)
w1 = torch.randn((2, 3, H, W), generator=g).double()
w2 = torch.randn((2, 20, H, W), generator=g).double()
taps = {}
P = {k: v.double() for k, v in P0.items()}
class T(dict):
    def __setitem__(self, k, v):
        v.retain_grad()
        super().__setitem__(k, v)
taps = T()
xin = torch.cat([x, seg], 1).double()
rr, sr = O.forward(P, xin, taps=taps) if False else (None, None)
# need grads: parameters not requiring grad -> make input require grad to build graph
xin.requires_grad_(True)
rr, sr = O.forward(P, xin, taps=taps)
((rr * w1).sum() + (sr * w2).sum()).backward()
rgb, s = m(x.to(dev), seg.to(dev))
((rgb * w1.float().to(dev)).sum() + (s * w2.float().to(dev)).sum()).backward()
torch.cuda.synchronize()
plan = [p for lst in m.coarse_model._pool.plans.values() for p in lst][0]
bufs = {b.name: b for b in plan.g.buffers}
for k, t in taps.items():
    ref = t.grad * torch.where(t > 0, 1.0, 0.2)  # pre-activation gradient (outputs are lrelu)
    got = bufs[k].g.detach().cpu().double().permute(0, 3, 1, 2)
    e = float((got - ref).abs().max()) / float(ref.abs().max())
    print(f"{k:40s} {e:.2e}{' <<<' if e > 1e-5 else ''}")
# sign-flip census: activations whose sign differs between the HIP fp32 plan and fp64
for k, t in taps.items():
    got = bufs[k].t.detach().cpu().double().permute(0, 3, 1, 2)
    flips = int(((got > 0) != (t.detach() > 0)).sum())
    gg = bufs[k].g.detach().cpu().double().permute(0, 3, 1, 2)
    ref = t.grad * torch.where(t > 0, 1.0, 0.2)
    l2 = float((gg - ref).norm() / ref.norm())
    if flips or l2 > 1e-5:
        print(f"{k:40s} sign flips {flips}  min|act| at flips {float(t.detach().abs()[(got > 0) != (t.detach() > 0)].max()) if flips else 0:.1e}  L2 rel {l2:.2e}")
