"""Time the weight-stationary 3x3 conv family (c, cout <= 64) through the C ABI under each
DVIE_CONV_STRIP mode (0 = tile kernel conv_ws, 1-3 = strip kernel variants), per
epilogue-operand set, with HIP events on the launch stream.

    python tools/conv_strip_micro.py [reps]

Prints per (shape, operands, mode): average launch time, TFLOP/s and the algorithmic HBM
rate (input + output + operand tensors once)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
lib = L.load()
stream = torch.cuda.current_stream()
sp = ctypes.c_void_p(stream.cuda_stream)
SHAPES = [(8, 256, 512, 64, 64), (16, 256, 512, 64, 64), (8, 256, 512, 32, 32)]
OPS = {"lrelu": (0, 0, 0, 1), "res+lrelu": (1, 0, 0, 1), "z": (0, 0, 1, 0), "beta+z": (0, 1, 1, 0)}

for n, H, W, c, cout in SHAPES:
    K = 9 * c
    kpad = (K + 63) // 64 * 64
    x = torch.randn(n, H, W, c, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, kpad, device=dev) / K ** 0.5).to(torch.bfloat16)
    y = torch.zeros(n, H, W, cout, device=dev, dtype=torch.bfloat16)
    r = torch.randn(n, H, W, cout, device=dev).to(torch.bfloat16)
    z = torch.randn(n, H, W, cout, device=dev).to(torch.bfloat16)
    flops = 2.0 * n * H * W * cout * c * 9
    for name, (res, beta, dz, act) in OPS.items():
        d = L.ConvDesc()
        d.x, d.w, d.y, d.bias = x.data_ptr(), w.data_ptr(), y.data_ptr(), None
        d.res = r.data_ptr() if res else None
        d.z = z.data_ptr() if dz else None
        d.x_ld, d.y_ld, d.res_ld, d.z_ld = c, cout, cout, cout
        d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, H, W, c, kpad, cout
        d.oh, d.ow, d.sy, d.sx = H, W, 1, 1
        d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = 3, 3, -1, -1, 1, 1
        d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = H, W, 1, 1, 0, 0
        d.act, d.dact, d.beta = act, L.ACT_LRELU if dz else 0, int(beta)
        d.dtype, d.out_f32, d.alpha = L.BF16, 0, 0.2
        nb = 2.0 * n * H * W * (c + cout * (1 + res + beta + dz))
        for mode in ("0", "1", "2", "3"):
            os.environ["DVIE_CONV_STRIP"] = mode
            for _ in range(3):
                L.check(lib.dvie_conv2d_fwd(ctypes.byref(d), sp), "conv")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                lib.dvie_conv2d_fwd(ctypes.byref(d), sp)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            print(f"{n}x{H}x{W} {c}->{cout} {name:10s} strip={mode} {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TFLOP/s  "
                  f"{nb / ms / 1e6:7.1f} GB/s", flush=True)
