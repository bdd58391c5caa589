"""Diagnostic: the attention-op chain of tests/test_gpu_refine.py buffer by buffer vs torch."""
import sys
sys.path.insert(0, ".")
import torch
from deep_video_interpolation_extrapolation_amd import engine as E
from oracle import refine as OR

dev = torch.device("cuda:0")
B, C, H, W = 2, 16, 7, 12
g = E.Graph(torch.float32)
X = {k: g.buffer(k, H, W, C) for k in ("x", "t1", "t2")}
for k, b in X.items():
    g.input_nchw(E.R(b), k, ext_c=C)
n = {k: g.buffer(k + "n", H, W, C) for k in X}
for k in X:
    g.l2norm(E.R(X[k]), E.R(n[k]))
sim = g.buffer("sim", H, W, 92)
g.corr(E.R(n["x"]), [E.R(n["t1"]), E.R(n["t2"])], E.R(sim), 5, 9)
prob = g.buffer("prob", H, W, 92)
g.softmax(E.R(sim), E.R(prob), 2, 5, 9)
out = g.buffer("out", H, W, C)
g.gather(E.R(prob), [E.R(X["t1"]), E.R(X["t2"])], E.R(out), 0, 2, 5, 9)
plan = g.compile(B, dev, backward=False)
gen = torch.Generator().manual_seed(4)
ins = {k: torch.randn((B, C, H, W), generator=gen) for k in X}
dins = {k: t.to(dev) for k, t in ins.items()}
for k, t in dins.items():
    plan.set_input(k, t)
plan.run_forward()
torch.cuda.synchronize()
nhwc = lambda b: b.t.cpu().double()
for k in X:
    print("in", k, float((nhwc(X[k]).permute(0, 3, 1, 2) - ins[k]).abs().max()))
    ref = ins[k] / ins[k].norm(dim=1, keepdim=True)
    print("norm", k, float((nhwc(n[k]).permute(0, 3, 1, 2) - ref).abs().max()))
r = {k: v.double() for k, v in ins.items()}
xn = r["x"] / r["x"].norm(dim=1, keepdim=True)
sims = []
for t in ("t1", "t2"):
    nb = OR._neighbours(r[t] / r[t].norm(dim=1, keepdim=True))
    sims.append(torch.stack([(xn * q).sum(1) for q in nb], -1))
simr = torch.cat(sims, -1)
print("sim", float((nhwc(sim)[..., :90] - simr).abs().max()))
print("sim[0,3,5,:12]", nhwc(sim)[0, 3, 5, :12].numpy().round(3), simr[0, 3, 5, :12].numpy().round(3))
pr = torch.softmax(simr, -1)
print("prob", float((nhwc(prob)[..., :90] - pr).abs().max()))
o = OR.weighted_neighbours(r["t1"], r["t2"], pr)
print("out", float((nhwc(out).permute(0, 3, 1, 2) - o).abs().max()))
