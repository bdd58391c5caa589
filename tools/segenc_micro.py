"""Segmentation-encoder fused backward micro-benchmark through the C ABI (dvie_segenc_bwd at
the bench shape, 8 x 256 x 512, synthetic bf16 maps), timed with HIP events per launch, under
each value of DVIE_SEGENC_DBG given on the command line (timing-only phase ablations read per
launch: 1 / 2 / 4 skip phase 1 / 2 / 3, 8 the tile loads, 16 the slab stores, 32 the tile loop;
0 = the real kernel).  The ablation bits exist only in the timing-only library
(-DDVIE_TIMING_DBG, results wrong; the product build ignores DVIE_SEGENC_DBG): copy that build
over the package's libdvie.so first, as tools/skip_ab.sh does.
usage: python tools/segenc_micro.py [dbg values ...]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402


def main():
    vals = sys.argv[1:] or ["0"]
    dev = torch.device("cuda:0")
    n, h, w = 8, 256, 512
    slabs = int(os.environ.get("SEGENC_SLABS", "256"))  # the launch's workgroups (one per CU)
    g = torch.Generator(device=dev).manual_seed(3)

    def bf(*shape):
        return (torch.rand(shape, generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    dout, e2, e1, inp = bf(n * h * w, 8), bf(n * h * w, 32), bf(n * h * w, 32), bf(n * h * w, 24)
    w4d, w2d = bf(32, 80), bf(32, 288)
    f = {k: torch.empty(slabs * m, device=dev) for k, m in
         (("dw4", 8 * 288), ("dw2", 32 * 288), ("dw0", 32 * 216), ("db4", 8), ("db2", 32), ("db0", 32))}
    d = L.SegencBwdDesc()
    d.dout, d.e2, d.e1, d.inp = dout.data_ptr(), e2.data_ptr(), e1.data_ptr(), inp.data_ptr()
    d.w4d, d.w2d = w4d.data_ptr(), w2d.data_ptr()
    for k, t in f.items():
        setattr(d, k, t.data_ptr())
    d.dout_ld, d.e2_ld, d.e1_ld, d.in_ld = 8, 32, 32, 24
    d.n, d.h, d.w, d.kpad4, d.kpad2, d.slabs = n, h, w, 80, 288, slabs
    lib = L.load()
    s = L.stream_ptr(dev)
    for v in vals:
        os.environ["DVIE_SEGENC_DBG"] = v
        for _ in range(3):
            L.check(lib.dvie_segenc_bwd(ctypes.byref(d), s), "segenc_bwd")
        torch.cuda.synchronize()
        e0, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            L.check(lib.dvie_segenc_bwd(ctypes.byref(d), s), "segenc_bwd")
        e1_.record()
        torch.cuda.synchronize()
        print(f"DVIE_SEGENC_DBG={v}: {e0.elapsed_time(e1_) / 20 * 1e3:.1f} us per launch", flush=True)
    os.environ.pop("DVIE_SEGENC_DBG")


if __name__ == "__main__":
    main()
