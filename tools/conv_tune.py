"""Time dvie_conv2d_fwd per tile configuration on HRNet-shaped convolutions and check each
result against torch's fp32 conv2d of the same bf16-rounded operands.

    python tools/conv_tune.py [cfgs] [iters] [shape-substring]   e.g.  python tools/conv_tune.py -1,0,1 20 '64->64'   (several: '128->128|256->256')
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402

SHAPES = [  # name, cin, cout, k, H, W, batch
    ("3x3 64->64 256x512", 64, 64, 3, 256, 512, 8),
    ("3x3 128->128 128x256", 128, 128, 3, 128, 256, 8),
    ("3x3 256->256 64x128", 256, 256, 3, 64, 128, 8),
    ("1x1 448->448 256x512", 448, 448, 1, 256, 512, 8),
    ("1x1 448->896 256x512", 448, 896, 1, 256, 512, 8),
    ("1x1 896->448 256x512", 896, 448, 1, 256, 512, 8),
    ("3x3 448->8 256x512 f32out", 448, 8, 3, 256, 512, 8),
    ("3x3 448->24 256x512", 448, 24, 3, 256, 512, 8),
    ("3x3 256->64 256x512", 256, 64, 3, 256, 512, 8),
    ("1x1 64->256 256x512", 64, 256, 1, 256, 512, 8),
    ("1x1 256->64 256x512", 256, 64, 1, 256, 512, 8),
    ("3x3 64->256 256x512", 64, 256, 3, 256, 512, 8),
    ("3x3 32->32 256x512", 32, 32, 3, 256, 512, 8),
    ("3x3 24->64 256x512", 24, 64, 3, 256, 512, 8),
    ("3x3 8->448 256x512", 8, 448, 3, 256, 512, 8),
    # VGG19's deep blocks (data gradients run on the 8 predicted frames, forwards on 16)
    ("3x3 512->512 16x32 b8", 512, 512, 3, 16, 32, 8),
    ("3x3 512->512 16x32 b16", 512, 512, 3, 16, 32, 16),
    ("3x3 512->512 32x64 b8", 512, 512, 3, 32, 64, 8),
    ("3x3 512->256 32x64 b8", 512, 256, 3, 32, 64, 8),
]


def main():
    cfgs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "-1,-3").split(",")]
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    only = sys.argv[3] if len(sys.argv) > 3 else ""
    lib = L.load()
    dev = torch.device("cuda:0")
    s = L.stream_ptr()
    first = True
    for name, cin, cout, k, H, W, B in SHAPES:
        if only and not any(o in name for o in only.split("|")):
            continue
        torch.manual_seed(0)
        out_f32 = "f32out" in name
        x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
        wt = (torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5).to(torch.bfloat16)
        kpad = (k * k * cin + 63) // 64 * 64
        wp = torch.zeros(cout, kpad, device=dev, dtype=torch.bfloat16)
        wp[:, :k * k * cin] = wt.permute(0, 2, 3, 1).reshape(cout, -1)
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), wt.float(), padding=k // 2).permute(0, 2, 3, 1)
        y = torch.empty(B, H, W, cout, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
        d = L.ConvDesc()
        d.x, d.w, d.y = x.data_ptr(), wp.data_ptr(), y.data_ptr()
        d.x_ld, d.y_ld = cin, cout
        d.n, d.ih, d.iw, d.c, d.kpad, d.cout = B, H, W, cin, kpad, cout
        d.oh, d.ow, d.sy, d.sx = H, W, 1, 1
        d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = k, k, -(k // 2), -(k // 2), 1, 1
        d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = H, W, 1, 1, 0, 0
        d.dtype, d.out_f32, d.alpha = L.BF16, int(out_f32), 0.2
        flops = 2.0 * B * H * W * cout * cin * k * k
        for cfg in cfgs:
            os.environ["DVIE_CONV_CFG"] = "" if cfg == -3 else str(cfg)
            y.zero_()
            rc = lib.dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(s))
            if rc:
                print(f"{name:28s} cfg {cfg:2d}: rc {rc} {lib.dvie_last_error()}")
                continue
            torch.cuda.synchronize()
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # warm-up long enough for the clocks to settle: with 3 launches the first config
            # timed in a process read ~8% slow (r01zd), which reorders close configs
            for _ in range(max(3, 4 * iters) if first else 3):
                lib.dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(s))
            e0.record()
            for _ in range(iters):
                lib.dvie_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(s))
            e1.record()
            torch.cuda.synchronize()
            first = False
            ms = e0.elapsed_time(e1) / iters
            print(f"{name:28s} cfg {cfg:2d}: {ms*1e3:8.1f} us  {flops/ms/1e9:7.1f} TF/s  relerr {err:.2e}"
                  f"{'  BAD' if err > 1e-2 else ''}", flush=True)
    os.environ.pop("DVIE_CONV_CFG", None)


if __name__ == "__main__":
    main()
