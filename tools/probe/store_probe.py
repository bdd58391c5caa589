"""Time tools/probe/store_probe.hip: the wide 1x1 epilogue's memory pattern (two bf16 operand
reads + one write, 256 channels per pixel) in the MFMA-layout order vs a coalesced order.
usage: python tools/probe/store_probe.py"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "store_probe.so"))
    dev = torch.device("cuda:0")
    npix = 8 * 256 * 512
    a = torch.randn(npix, 256, device=dev).to(torch.bfloat16)
    b = torch.randn(npix, 256, device=dev).to(torch.bfloat16)
    ys = [torch.empty_like(a) for _ in range(3)]
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for mode in (0, 1, 2, 0, 1, 2):
        y = ys[mode]
        for _ in range(5):
            lib.store_probe(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                            ctypes.c_longlong(npix), mode, s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            lib.store_probe(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                            ctypes.c_longlong(npix), mode, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"mode {mode}: {ms * 1e3:.1f} us  {3 * a.numel() * 2 / ms / 1e6:.0f} GB/s", flush=True)
    # (the probe's pixels are 16 groups of 16 B = 128 bf16 channels: the first half of each buffer)
    half = ys[0].view(torch.int16).flatten()[: npix * 128]
    assert torch.equal(half, ys[1].view(torch.int16).flatten()[: npix * 128])


if __name__ == "__main__":
    main()
