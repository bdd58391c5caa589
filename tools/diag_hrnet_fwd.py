"""Diagnostic: compare every stage-branch activation buffer of the HIP plan with the
oracle's, after forward and again after backward (detects clobbered buffers)."""
import os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
os.environ["DVIE_PRECISION"] = "fp32"
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
taps = {}
with torch.no_grad():
    rr, sr = O.forward({k: v.double() for k, v in P0.items()}, torch.cat([x, seg], 1).double(), taps=taps)
rgb, s = m(x.to(dev), seg.to(dev))
torch.cuda.synchronize()
print("fwd out err", float((rgb.detach().cpu().double() - rr).abs().max()), float((s.detach().cpu().double() - sr).abs().max()))
plan = [p for lst in m.coarse_model._pool.plans.values() for p in lst][0]
bufs = {b.name: b for b in plan.g.buffers}
def report(tag):
    for k, ref in taps.items():
        b = bufs[k]
        got = b.t.detach().cpu().double().permute(0, 3, 1, 2)
        e = float((got - ref).abs().max()) / float(ref.abs().max())
        print(f"{tag} {k:40s} {e:.2e}{' <<<' if e > 1e-5 else ''}")
report("after-fwd")
(rgb.sum() + s.sum()).backward()
torch.cuda.synchronize()
report("after-bwd")
