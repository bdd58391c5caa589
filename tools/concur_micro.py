"""Do HRNet's independent branch convs gain from running on two HIP streams at once?
Builds one conv plan per branch shape (3x3, residual-free, LeakyReLU, bf16, batch 8: the
stage-3 branches 64ch@256x512 / 128ch@128x256 / 256ch@64x128) and times, with HIP events,
`iters` forwards (or forward+backward) of each plan alone, all plans one after the other on
one stream, and each plan on its own stream at the same time.
    python tools/concur_micro.py [iters] [bwd]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402
from deep_video_interpolation_extrapolation_amd import engine as E  # noqa: E402
from deep_video_interpolation_extrapolation_amd.nets.conv import Conv2d  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
bwd = len(sys.argv) > 2 and sys.argv[2] == "bwd"
dev = torch.device("cuda:0")
B = 8


def make(c, H, W, nconv=2):
    ms = [Conv2d(c, c, 3, 1, 1, bias=False).to(dev) for _ in range(nconv)]
    g = E.Graph(torch.bfloat16)
    bufs = [g.buffer(f"x{i}", H, W, c) for i in range(nconv + 1)]
    g.input_nchw(E.R(bufs[0]), "in", ext_c=c, requires_grad=False)
    for i, m in enumerate(ms):
        g.conv(E.R(bufs[i]), m, E.R(bufs[i + 1]), act=L.ACT_LRELU, name=f"conv{i}")
    mo = Conv2d(c, 8, 1, 1, 0, bias=False).to(dev)
    zb = g.buffer("z", H, W, 8, dtype=torch.float32, external=True)
    g.conv(E.R(bufs[-1]), mo, E.R(zb), name="post")
    g.output("z", E.R(zb), 8)
    plan = g.compile(B, dev, backward=bwd)
    plan.set_input("in", torch.randn(B, c, H, W, device=dev))
    plan.set_output("z", torch.empty(B, H, W, 8, device=dev))
    if bwd:
        plan.set_output_grad("z", torch.randn(B, 8, H, W, device=dev))
        for m in ms + [mo]:
            m.weight.grad = torch.zeros_like(m.weight)
        plan.set_param_grads(True)
    return plan


plans = {"b0 64@256x512": make(64, 256, 512), "b1 128@128x256": make(128, 128, 256),
         "b2 256@64x128": make(256, 64, 128)}
streams = {k: torch.cuda.Stream(device=dev) for k in plans}


def step(plan, s):
    plan.run_forward(stream=s)
    if bwd:
        plan.run_backward(stream=s)


def timed(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    # every stream's work is ordered before e1 through waits on the default stream
    for s in streams.values():
        torch.cuda.current_stream().wait_stream(s)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


cur = L.stream_ptr()
for k, p in plans.items():  # warm-up
    step(p, cur)
alone = {}
for k, p in plans.items():
    alone[k] = timed(lambda: [step(p, cur) for _ in range(iters)])
    print(f"{k}: {alone[k] * 1e3:.1f} us/iter alone", flush=True)
for names in (list(plans), list(plans)[1:], list(plans)[:2]):
    seq = timed(lambda: [step(plans[k], cur) for _ in range(iters) for k in names])

    def conc():
        for s in streams.values():
            s.wait_stream(torch.cuda.current_stream())
        for _ in range(iters):
            for k in names:
                step(plans[k], streams[k].cuda_stream)
    par = timed(conc)
    print(f"{' + '.join(names)}: one stream {seq * 1e3:.1f} us/iter, own streams {par * 1e3:.1f} us/iter "
          f"({(seq - par) / seq * 100:+.1f}% saved)", flush=True)
