"""1x1 conv (dvie_conv2d_fwd, NHWC) vs the library GEMM (torch.matmul -> hipBLASLt) on the
same operands: Y[px, co] = X[px, ci] . W[co, ci]^T, bf16, fp32 accumulation.

    python tools/gemm_vs_blas.py [reps]

Prints per shape: our 1x1 launch (plain + LeakyReLU epilogue) and the library GEMM (no
epilogue) in us and TFLOP/s, HIP events on the current stream."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
lib = L.load()
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
SHAPES = [(8, 256, 512, 448, 896), (8, 256, 512, 896, 448), (8, 256, 512, 448, 448), (8, 256, 512, 64, 256),
          (8, 256, 512, 256, 64), (8, 128, 256, 256, 128)]


def tm(fn):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for n, H, W, c, cout in SHAPES:
    M = n * H * W
    x = torch.randn(M, c, device=dev).to(torch.bfloat16)
    kpad = (c + 63) // 64 * 64
    w = (torch.randn(cout, kpad, device=dev) / c ** 0.5).to(torch.bfloat16)
    y = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    d = L.ConvDesc()
    d.x, d.w, d.y, d.bias, d.res, d.z = x.data_ptr(), w.data_ptr(), y.data_ptr(), None, None, None
    d.x_ld, d.y_ld, d.res_ld, d.z_ld = c, cout, cout, cout
    d.n, d.ih, d.iw, d.c, d.kpad, d.cout = n, H, W, c, kpad, cout
    d.oh, d.ow, d.sy, d.sx = H, W, 1, 1
    d.th, d.tw, d.dy0, d.dx0, d.ddy, d.ddx = 1, 1, 0, 0, 1, 1
    d.yh, d.yw, d.osy, d.osx, d.ory, d.orx = H, W, 1, 1, 0, 0
    d.act, d.dact, d.beta = L.ACT_LRELU, 0, 0
    d.dtype, d.out_f32, d.alpha = L.BF16, 0, 0.2
    ms_ours = tm(lambda: lib.dvie_conv2d_fwd(ctypes.byref(d), sp))
    wt = w[:, :c].t().contiguous()
    yb = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
    ms_blas = tm(lambda: torch.matmul(x, wt, out=yb))
    ms_blas_t = tm(lambda: torch.matmul(x, w[:, :c].t(), out=yb))
    fl = 2.0 * M * c * cout
    print(f"{M}x{c}->{cout}: ours {ms_ours * 1e3:8.1f} us {fl / ms_ours / 1e9:7.1f} TF/s | blas NN {ms_blas * 1e3:8.1f} us "
          f"{fl / ms_blas / 1e9:7.1f} TF/s | blas NT {ms_blas_t * 1e3:8.1f} us {fl / ms_blas_t / 1e9:7.1f} TF/s", flush=True)
