"""Diagnostic: for every stride-1 dgrad CONV op of the HRNet backward, recompute its output
on the host from the device buffers it reads, and check its packed weights."""
import ctypes, os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
os.environ["DVIE_PRECISION"] = "fp32"
import torch
import torch.nn.functional as F
import inputs
from deep_video_interpolation_extrapolation_amd import nets, _lib as L, engine as E

dev = torch.device("cuda:0")
torch.manual_seed(1024)
m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet")).to(dev)
x, seg = inputs.hrnet_input(2, 32, 64)
rgb, s = m(x.to(dev), seg.to(dev))
(rgb.square().sum() + s.square().sum()).backward()
torch.cuda.synchronize()
plan = [p for lst in m.coarse_model._pool.plans.values() for p in lst][0]
g = plan.g
# map grad-buffer pointer -> buffer
gb = {b.g.data_ptr(): b for b in g.buffers if b.g is not None}
# walk ConvOps: find the dgrad emitted for each conv with a stride-1 layer
bad = 0
for op in g.ops:
    if not isinstance(op, E.ConvOp) or op.layer.stride != 1 or not op.x.buf.needs_grad:
        continue
    lay = op.layer
    if op.x.buf.g is None or op.out.buf.g is None or op.out.buf.external:
        continue
    (ph, wt, kpad), = [v for k, v in lay.wd][0]
    # expected packed dgrad weights: [cin_p][t*cout_p + co] = W[co][cmap[r]][kh][kw]
    W = lay.m.weight.detach()
    exp = torch.zeros(lay.cin_p, kpad, device=dev)
    T = lay.kh * lay.kw
    for r in range(lay.cin_p):
        ci = lay.cmap[r]
        if ci < 0: continue
        for t in range(T):
            kh, kw = t // lay.kw, t % lay.kw
            exp[r, t * lay.cout_p: t * lay.cout_p + lay.cout] = W[:, ci, kh, kw]
    werr = float((wt.float() - exp).abs().max())
    # expected output (pre-activation grad of x region, only valid if x has one contribution)
    gout = op.out.buf.g[..., op.out.c0: op.out.c0 + lay.cout].permute(0, 3, 1, 2).double()
    ref = torch.nn.grad.conv2d_input((gout.shape[0], lay.cin, op.x.H, op.x.W), W.double(), gout, padding=lay.pad)
    xb = op.x.buf
    single = xb.expected == 1 and len(xb.producers) == 1 and xb.producers[0].act == 1
    if single:
        z = xb.t[..., op.x.c0: op.x.c0 + lay.cin].permute(0, 3, 1, 2).double()
        ref = ref * torch.where(z > 0, 1.0, 0.2)
        got = xb.g[..., op.x.c0: op.x.c0 + lay.cin].permute(0, 3, 1, 2).double()
        e = float((got - ref).abs().max() / ref.abs().max())
    else:
        e = float("nan")
    flag = " <<<" if (werr > 0 or e > 1e-5) else ""
    if flag: bad += 1
    print(f"{lay.name:45s} werr={werr:.1e} out_err={e:.2e} {tuple(op.x.buf.g.shape)}{flag}")
print("bad", bad)
