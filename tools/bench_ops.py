"""Per-op microbenchmark of the plan kernels on HRNet-shaped convolutions.

    python tools/bench_ops.py [bf16|fp32] [batch]

For each representative layer shape (HRNet @256x512) builds a one-conv graph whose input
is an internal NHWC buffer and whose output feeds a second conv (so dgrad/wgrad are on
the same footing as inside HRNet), runs forward+backward plans a few times with per-op
HIP events (engine.PROFILE) and prints time / TFLOP/s / GB/s per op class.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402
from deep_video_interpolation_extrapolation_amd import engine as E  # noqa: E402
from deep_video_interpolation_extrapolation_amd.nets.conv import Conv2d  # noqa: E402

SHAPES = [  # name, cin, cout, k, stride, H, W
    ("3x3 64->64 full", 64, 64, 3, 1, 256, 512),
    ("1x1 256->64 full", 256, 64, 1, 1, 256, 512),
    ("1x1 64->256 full", 64, 256, 1, 1, 256, 512),
    ("3x3 128->128 half", 128, 128, 3, 1, 128, 256),
    ("3x3 256->256 quarter", 256, 256, 3, 1, 64, 128),
    ("3x3 s2 64->128", 64, 128, 3, 2, 256, 512),
    ("1x1 448->448 full", 448, 448, 1, 1, 256, 512),
    ("3x3 448->8 full (head)", 448, 3, 3, 1, 256, 512),
]


def run(prec, batch, reps=5):
    dt = torch.bfloat16 if prec == "bf16" else torch.float32
    dev = torch.device("cuda:0")
    rows = []
    for name, cin, cout, k, s, H, W in SHAPES:
        torch.manual_seed(0)
        m = Conv2d(cin, cout, k, s, k // 2, bias=False).to(dev)
        m2 = Conv2d(E.rup(cout, 8), 8, 1, 1, 0, bias=False).to(dev)
        g = E.Graph(dt)
        xb = g.buffer("x", H, W, cin)
        oh, ow = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
        yb = g.buffer("y", oh, ow, E.rup(cout, 8))
        # x is produced by a conv so it needs a gradient (dgrad is exercised)
        x0 = g.buffer("x0", H, W, 8)
        m0 = Conv2d(8, cin, 1, 1, 0, bias=False).to(dev)
        g.input_nchw(E.R(x0), "in", ext_c=8)
        g.conv(E.R(x0), m0, E.R(xb), act=L.ACT_LRELU, name="pre")
        g.conv(E.R(xb), m, E.R(yb), act=L.ACT_LRELU, name="conv")
        zb = g.buffer("z", oh, ow, 8, dtype=torch.float32, external=True)
        g.conv(E.R(yb), m2, E.R(zb), name="post")
        g.output("z", E.R(zb), 8)
        plan = g.compile(batch, dev, backward=True)
        inp = torch.randn(batch, 8, H, W, device=dev)
        plan.set_input("in", inp)
        z = torch.empty(batch, oh, ow, 8, device=dev)
        plan.set_output("z", z)
        gz = torch.randn(batch, 8, oh, ow, device=dev)
        plan.set_output_grad("z", gz)
        for p in (m, m0, m2):
            p.weight.grad = torch.zeros_like(p.weight)
        plan.set_param_grads(True)
        for _ in range(2):
            plan.run_forward()
            plan.run_backward()
        torch.cuda.synchronize()
        prof = []
        E.PROFILE = prof
        for _ in range(reps):
            plan.run_forward()
            plan.run_backward()
        torch.cuda.synchronize()
        E.PROFILE = None
        agg = {}
        for meta, kind, e0, e1 in prof:
            if not meta or meta.get("name") != "conv":
                if kind == L.OP_WREDUCE or kind == L.OP_COLSUM:
                    agg.setdefault("reduce", [0.0, 0.0, 0.0])[0] += e0.elapsed_time(e1)
                continue
            a = agg.setdefault(meta["cls"], [0.0, 0.0, 0.0])
            a[0] += e0.elapsed_time(e1)
            a[1] += meta["flops"]
            a[2] += meta["bytes"]
        for cls, (ms, fl, by) in sorted(agg.items()):
            ms /= reps
            fl /= reps
            by /= reps
            rows.append((name, cls, ms, fl / ms / 1e9 if fl else 0.0, by / ms / 1e6 if by else 0.0))
        del plan
    print(f"{'shape':28s} {'op':11s} {'ms':>8s} {'TFLOP/s':>9s} {'GB/s':>8s}")
    for r in rows:
        print(f"{r[0]:28s} {r[1]:11s} {r[2]:8.3f} {r[3]:9.1f} {r[4]:8.1f}")


if __name__ == "__main__":
    run(sys.argv[1] if len(sys.argv) > 1 else "bf16", int(sys.argv[2]) if len(sys.argv) > 2 else 8)
