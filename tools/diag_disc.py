"""Diagnostics: where do the HIP discriminator gradients differ from the fp64 oracle?
Prints, per input and per parameter, relative L2 vs fp64 for HIP and for the fp32 CPU
oracle, plus how concentrated the HIP error is (a LeakyReLU kink flip is local: a few
large-error pixels; a systematic error is diffuse)."""
import os
import sys
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
os.environ["DVIE_PRECISION"] = "fp32"

import inputs  # noqa: E402
from oracle import disc as OD  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


def main(kind="frame", seed=31, H=128, W=128):
    from deep_video_interpolation_extrapolation_amd import nets
    dev = torch.device("cuda:0")
    torch.manual_seed(seed)
    cls = nets.FrameDiscriminator if kind == "frame" else nets.VideoDiscriminator
    d = cls(types.SimpleNamespace(seg_disc=True, precision="fp32")).to(dev)
    spec = (OD.FRAME if kind == "frame" else OD.VIDEO)(23)
    P = OD.init_params(spec, seed)
    x, seg, ix, iseg, gout = inputs.disc_inputs(2, H, W)
    ins = [x, seg] + ([ix, iseg] if kind == "video" else [])

    def oracle(dt):
        st = {k[:-len(".running_mean")]: (P[k].clone().to(dt), P[k[:-4] + "var"].clone().to(dt))
              for k in P if k.endswith("running_mean")}
        oi = [v.clone().to(dt).requires_grad_(True) for v in ins]
        pr = {k: v.clone().to(dt).requires_grad_(True) for k, v in P.items() if "running" not in k}
        r = OD.forward(pr, spec, torch.cat(oi, 1), training=True, stats=st)
        r.backward(gout.to(dt))
        return r, oi, pr

    r32, i32, p32 = oracle(torch.float32)
    r64, i64, p64 = oracle(torch.float64)
    gi = [v.to(dev).requires_grad_(True) for v in ins]
    out = d(*gi)
    out.backward(gout.to(dev))
    torch.cuda.synchronize()
    print(f"{kind} {H}x{W} score: hip {rel(out.detach(), r64.detach()):.2e} cpu32 {rel(r32.detach(), r64.detach()):.2e}")
    for k, (a, b, c) in enumerate(zip(gi, i32, i64)):
        dd = (a.grad.double().cpu() - c.grad.double()).abs()
        thr = 1e-3 * float(c.grad.abs().max())
        n_big = int((dd > thr).sum())
        pos = (dd > thr).nonzero()[:8].tolist()
        print(f"  input {k}: hip {rel(a.grad, c.grad):.2e} cpu32 {rel(b.grad, c.grad):.2e}  "
              f"elements > 1e-3*max: {n_big} / {dd.numel()}  first at {pos}")
    named = dict(d.named_parameters())
    for k in p64:
        print(f"  {k:24s} hip {rel(named[k].grad, p64[k].grad):.2e} cpu32 {rel(p32[k].grad, p64[k].grad):.2e}")


if __name__ == "__main__":
    main("frame", 31, 128, 128)
    main("video", 32, 128, 256)
