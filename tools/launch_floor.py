"""Launch floor of an empty kernel (dvie_launch_probe) per grid shape: `reps` launches replayed
from a captured hipGraph, HIP-event time per launch.  usage: python tools/launch_floor.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_video_interpolation_extrapolation_amd import _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lib = L.load()
    for blocks, threads in ((1024, 256), (512, 512), (256, 1024), (4096, 256), (2048, 512), (1024, 1024), (256, 256)):
        def fn():
            L.check(lib.dvie_launch_probe(blocks, threads, L.stream_ptr(dev)), "probe")
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(50):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"{blocks} x {threads}: {e0.elapsed_time(e1) / 50 * 1e3:.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
