"""Stress-check every weight-gradient launch of the full-size InterNet plan: fresh random
operands, slab workspace pre-filled with NaN plus a guard zone, then (1) the guard is intact,
(2) every slab entry the reduction reads is finite, (3) the reduced gradient matches torch.
    python tools/wgrad_check.py [batch]"""
import ctypes
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L, engine as E, nets  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda", 0)
    lib = L.load()
    s = ctypes.c_void_p(L.stream_ptr())
    torch.manual_seed(1024)
    m = nets.InterNet(types.SimpleNamespace(syn_type="inter", highres_large=False, coarse_model="HRNet")).to(dev)
    g = m.coarse_model._lower(E.Graph(torch.bfloat16), 256, 512)
    plan = g.compile(B, dev, backward=True)
    seen = set()
    bad = 0
    for i in range(plan.n_bwd):
        o = plan.bwd_arr[i]
        if o.kind != L.OP_WGRAD:
            continue
        d0 = o.u.wgrad
        key = (d0.n, d0.oh, d0.ow, d0.cout, d0.ih, d0.iw, d0.c, d0.sy, d0.th, d0.tw, d0.dy0, d0.dx0, d0.g_ld, d0.x_ld)
        if key in seen:
            continue
        seen.add(key)
        d = L.WgradDesc()
        ctypes.memmove(ctypes.addressof(d), ctypes.addressof(d0), ctypes.sizeof(d))
        gt = (torch.randn(d.n * d.oh * d.ow * d.g_ld, device=dev) * 0.1).to(torch.bfloat16)
        xt = torch.randn(d.n * d.ih * d.iw * d.x_ld, device=dev).to(torch.bfloat16)
        slabs = lib.dvie_wgrad_slabs(ctypes.byref(d))
        ntap = d.th * d.tw
        n_ws = slabs * d.cout * ntap * d.c
        ws = torch.full((n_ws + 4096,), float("nan"), device=dev)
        ws[n_ws:] = 12345.0
        d.g, d.x, d.ws = gt.data_ptr(), xt.data_ptr(), ws.data_ptr()
        L.check(lib.dvie_conv2d_wgrad(ctypes.byref(d), s), "wgrad")
        torch.cuda.synchronize()
        guard_ok = bool((ws[n_ws:] == 12345.0).all())
        part = ws[:n_ws].view(slabs, d.cout, ntap, d.c)
        finite = bool(torch.isfinite(part).all())
        # reference: sum over pixels of g[pix][co] * x[pix + tap][ci]
        G = gt.float().view(d.n, d.oh, d.ow, d.g_ld)[..., :d.cout].permute(0, 3, 1, 2)
        X = xt.float().view(d.n, d.ih, d.iw, d.x_ld)[..., :d.c].permute(0, 3, 1, 2)
        ref = torch.zeros(d.cout, ntap, d.c, device=dev)
        Xp = torch.nn.functional.pad(X, (8, 8, 8, 8))
        for t in range(ntap):
            ti, tj = t // d.tw, t % d.tw
            dy, dx = d.dy0 + ti * d.ddy, d.dx0 + tj * d.ddx
            ys = torch.arange(d.oh, device=dev) * d.sy + dy + 8
            xs = torch.arange(d.ow, device=dev) * d.sx + dx + 8
            Xs = Xp[:, :, ys][:, :, :, xs]
            ref[:, t, :] = torch.einsum("nchw,nkhw->ck", G, Xs)
        got = part.sum(0) if finite else None
        err = float((got - ref).abs().max() / ref.abs().max()) if finite else float("nan")
        ok = guard_ok and finite and err < 1e-3
        bad += not ok
        print(f"{'OK ' if ok else 'BAD'} n{d.n} {d.oh}x{d.ow} c{d.c}->{d.cout} taps {d.th}x{d.tw} s{d.sy} "
              f"g_ld{d.g_ld} x_ld{d.x_ld} splits {d.splits} slabs {slabs}: guard {guard_ok} finite {finite} "
              f"relerr {err:.2e}", flush=True)
    print("bad", bad)


if __name__ == "__main__":
    main()
