"""Flow-warp micro-benchmark through the C ABI (for rocprofv3 --kernel-trace --stats).

Runs dvie_warp_fwd / dvie_warp_bwd (and the dflow-only backward) on the bench's smooth
flow field at 8x3x256x512 and 8x3x1024x2048, `--reps` times each, and prints the
HIP-event time per call.  usage: python tools/warp_micro.py [--reps 50]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402


def setup(dev, n, c, H, W):
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.rand((n, c, H, W), generator=g, device=dev)
    yy, xx = torch.meshgrid(torch.linspace(0, 1, H, device=dev), torch.linspace(0, 1, W, device=dev), indexing="ij")
    flow = torch.stack([torch.sin(6.3 * xx + 3.1 * yy) * 0.016, torch.cos(4.7 * yy - 2.9 * xx) * 0.024])
    flow = flow.unsqueeze(0).repeat(n, 1, 1, 1) + (torch.rand((n, 2, H, W), generator=g, device=dev) - 0.5) * 4e-4
    go = torch.randn((n, c, H, W), generator=g, device=dev)
    out, dx, dflow = torch.empty_like(x), torch.zeros_like(x), torch.empty_like(flow)
    lib = L.load()
    d = L.WarpDesc()
    d.img, d.flow, d.out, d.dout, d.dimg, d.dflow = (t.data_ptr() for t in (x, flow, out, go, dx, dflow))
    d.n, d.c, d.h, d.w, d.align_corners = n, c, H, W, 1
    ws = torch.empty(lib.dvie_warp_ws_floats(ctypes.byref(d)), device=dev)
    d.ws = ws.data_ptr()
    return lib, d, (x, flow, go, out, dx, dflow, ws)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--shape", default=None, help="one n,c,H,W shape instead of the two defaults")
    a = ap.parse_args()
    shapes = [tuple(map(int, a.shape.split(",")))] if a.shape else [(8, 3, 256, 512), (8, 3, 1024, 2048)]
    dev = torch.device("cuda:0")
    s = L.stream_ptr(dev)
    for (n, c, H, W) in shapes:
        lib, d, keep = setup(dev, n, c, H, W)
        dx = keep[4]
        for tag in ("fwd", "bwd", "bwd_dflow_only"):
            d.dimg = None if tag == "bwd_dflow_only" else dx.data_ptr()

            def run():
                if tag == "fwd":
                    L.check(lib.dvie_warp_fwd(ctypes.byref(d), s), tag)
                else:
                    L.check(lib.dvie_warp_bwd(ctypes.byref(d), s), tag)
            for _ in range(3):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            msg = f"{n}x{c}x{H}x{W} {tag}: {e0.elapsed_time(e1) / a.reps * 1e3:.1f} us/call"
            if tag != "fwd":  # bit-level digest of the gradients (A/B runs of kernel variants)
                import hashlib
                h = hashlib.sha1()
                for t in ((keep[5],) if tag == "bwd_dflow_only" else (dx, keep[5])):
                    h.update(t.cpu().numpy().tobytes())
                msg += f" digest {h.hexdigest()[:16]}"
            print(msg, flush=True)


if __name__ == "__main__":
    main()
