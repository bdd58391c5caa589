"""Time dvie_conv2d_wgrad (+ dvie_wgrad_reduce) on HRNet-shaped convolutions and check the
weight gradient against torch's fp32 conv2d_weight of the same bf16-rounded operands.

    python tools/wgrad_tune.py [iters] [shape-substring] [force-per-tap]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402

if os.environ.get("DVIE_TOOL_LIB"):  # e.g. a -DDVIE_TIMING_DBG build for DVIE_WG_DBG ablations
    L.LIB_PATH = os.environ["DVIE_TOOL_LIB"]

SHAPES = [  # name, cin, cout, k, H, W, batch
    ("3x3 64->64 256x512", 64, 64, 3, 256, 512, 8),
    ("3x3 128->128 128x256", 128, 128, 3, 128, 256, 8),
    ("3x3 256->256 64x128", 256, 256, 3, 64, 128, 8),
    ("1x1 448->448 256x512", 448, 448, 1, 256, 512, 8),
    ("3x3 256->64 256x512", 256, 64, 3, 256, 512, 8),
    ("1x1 64->256 256x512", 64, 256, 1, 256, 512, 8),
    ("1x1 256->64 256x512", 256, 64, 1, 256, 512, 8),
    ("3x3 32->32 256x512", 32, 32, 3, 256, 512, 8),
    ("3x3 24->64 256x512", 24, 64, 3, 256, 512, 8),
    ("3x3 448->8 256x512", 448, 8, 3, 256, 512, 8),
    ("3x3 448->24 256x512", 448, 24, 3, 256, 512, 8),
]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    only = sys.argv[2] if len(sys.argv) > 2 else ""
    lib = L.load()
    dev = torch.device("cuda:0")
    s = L.stream_ptr()
    for name, cin, cout, k, H, W, B in SHAPES:
        if only and not any(o in name for o in only.split("|")):
            continue
        torch.manual_seed(0)
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        g = (torch.randn(B, H, W, cout, device=dev) * 0.1).to(torch.bfloat16)
        ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (cout, cin, k, k),
                                          g.float().permute(0, 3, 1, 2), padding=k // 2)
        d = L.WgradDesc()
        d.g, d.x = g.data_ptr(), x.data_ptr()
        d.g_ld, d.x_ld = cout, cin
        d.n, d.oh, d.ow, d.cout = B, H, W, cout
        d.ih, d.iw, d.c, d.sy, d.sx = H, W, cin, 1, 1
        d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = k, k, -(k // 2), -(k // 2), 1, 1
        d.dtype = L.BF16
        hint = lib.dvie_wgrad_splits_hint(ctypes.byref(d))
        d.splits = hint if hint > 0 else 64
        slabs = lib.dvie_wgrad_slabs(ctypes.byref(d))
        ws = torch.empty(slabs * cout * k * k * cin, device=dev)
        d.ws = ws.data_ptr()
        dw = torch.zeros(cout, cin, k, k, device=dev)
        r = L.WreduceDesc()
        r.ws, r.dw, r.cmap = ws.data_ptr(), dw.data_ptr(), None
        r.splits, r.ws_rows, r.ws_k, r.co_off = slabs, cout, k * k * cin, 0
        r.cout_p, r.cin_p, r.kh_n, r.kw_n, r.c, r.beta = cout, cin, k, k, cin, 0

        def run():
            L.check(lib.dvie_conv2d_wgrad(ctypes.byref(d), ctypes.c_void_p(s)), "wgrad")
            L.check(lib.dvie_wgrad_reduce(ctypes.byref(r), ctypes.c_void_p(s)), "wreduce")

        run()
        torch.cuda.synchronize()
        err = ((dw - ref).abs().max() / ref.abs().max()).item()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        ev[0].record()
        for _ in range(iters):
            lib.dvie_conv2d_wgrad(ctypes.byref(d), ctypes.c_void_p(s))
        ev[1].record()
        for _ in range(iters):
            lib.dvie_wgrad_reduce(ctypes.byref(r), ctypes.c_void_p(s))
        ev[2].record()
        torch.cuda.synchronize()
        t1 = ev[0].elapsed_time(ev[1]) / iters
        t2 = ev[1].elapsed_time(ev[2]) / iters
        flops = 2.0 * B * H * W * cout * cin * k * k
        print(f"{name:24s} splits {d.splits:4d} slabs {slabs:4d}: wgrad {t1*1e3:8.1f} us ({flops/t1/1e9:6.1f} TF/s)"
              f"  reduce {t2*1e3:7.1f} us  relerr {err:.2e}{'  BAD' if err > 1e-2 else ''}", flush=True)


if __name__ == "__main__":
    main()
