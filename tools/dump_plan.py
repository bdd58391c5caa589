"""Dump the HRNet backward descriptor list (CPU, no launch): op kind, target and sources."""
import os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch
from deep_video_interpolation_extrapolation_amd import nets, engine as E, _lib as L
torch.manual_seed(1024)
m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet"))
hr = m.coarse_model
g = hr._lower(E.Graph(torch.float32), 32, 64)
plan = g.compile(2, torch.device("cpu"), backward=True)
regions = []
for b in g.buffers:
    if b.g is not None: regions.append(("G:" + b.name, b.g))
    if b.t is not None: regions.append(("A:" + b.name, b.t))
def owner(ptr):
    if not ptr: return "-"
    for n, t in regions:
        if t.data_ptr() <= ptr < t.data_ptr() + t.numel() * t.element_size():
            return n
    return "?"
pat = sys.argv[1] if len(sys.argv) > 1 else ""
for i in range(plan.n_bwd):
    o = plan.bwd_arr[i]
    if o.kind == L.OP_CONV:
        d = o.u.conv
        s = f"CONV y={owner(d.y)} x={owner(d.x)} res={owner(d.res)} z={owner(d.z)} beta={d.beta} dact={d.dact} ph=({d.ory},{d.orx})"
    elif o.kind == L.OP_EW:
        d = o.u.ew
        s = f"EW{d.op} y={owner(d.y)} s0={owner(d.src0)} s1={owner(d.src1)} res={owner(d.res)} z={owner(d.z)} beta={d.beta} dact={d.dact}"
    elif o.kind == L.OP_WGRAD:
        d = o.u.wgrad
        s = f"WGRAD g={owner(d.g)} x={owner(d.x)}"
    else:
        s = f"kind{o.kind}"
    if pat in s:
        print(i, s)
