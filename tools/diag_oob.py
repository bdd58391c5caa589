"""Diagnostic: execute the HRNet backward op list one descriptor at a time and report any
op that changes a gradient/activation buffer other than the one it targets."""
import ctypes, os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
os.environ["DVIE_PRECISION"] = "fp32"
import torch
import inputs
from deep_video_interpolation_extrapolation_amd import nets, _lib as L

dev = torch.device("cuda:0")
torch.manual_seed(1024)
m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet")).to(dev)
x, seg = inputs.hrnet_input(2, 32, 64)
rgb, s = m(x.to(dev), seg.to(dev))
plan = [p for lst in m.coarse_model._pool.plans.values() for p in lst][0]
hr = m.coarse_model
hr.grad_views()
plan.set_param_grads(False)
g1 = torch.randn_like(rgb); g2 = torch.randn_like(s)
plan.set_output_grad("rgb", g1); plan.set_output_grad("segout", g2)
torch.cuda.synchronize()
regions = []
for b in plan.g.buffers:
    if b.g is not None:
        regions.append(("G:" + b.name, b.g))
    if b.t is not None:
        regions.append(("A:" + b.name, b.t))
def snap():
    return [float(t.double().abs().sum()) for _, t in regions]
def target(o):
    k = o.kind
    if k == L.OP_CONV: return o.u.conv.y
    if k == L.OP_EW: return o.u.ew.y
    return None
def owner(ptr):
    for n, t in regions:
        if t.data_ptr() <= ptr < t.data_ptr() + t.numel() * t.element_size():
            return n
    return "?"
lib = L.load()
stream = L.stream_ptr()
base = ctypes.addressof(plan.bwd_arr)
sz = ctypes.sizeof(L.Op)
prev = snap()
bad = 0
for i in range(plan.n_bwd):
    o = plan.bwd_arr[i]
    L.check(lib.dvie_run_ops(base + i * sz, 1, stream), f"op {i}")
    torch.cuda.synchronize()
    cur = snap()
    tgt = target(o)
    tname = owner(tgt) if tgt else None
    changed = [regions[j][0] for j in range(len(regions)) if cur[j] != prev[j]]
    extra = [c for c in changed if c != tname]
    if extra:
        bad += 1
        print(f"op {i} kind {o.kind} target {tname}: also changed {extra}")
    prev = cur
print("ops with foreign writes:", bad, "of", plan.n_bwd)
