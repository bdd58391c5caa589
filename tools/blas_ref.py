"""Vendor-library reference points for the hand-written conv kernels (tools/conv_tune.py
times those on the same shapes): torch.mm (hipBLASLt) on the 1x1-conv GEMM shapes of the
HRNet heads and bottlenecks, and torch's conv2d (MIOpen) in channels-last bf16 on the 3x3
shapes of the HRNet branches and heads."""
import sys
import torch

CONVS = [  # name, cin, cout, H, W, batch (3x3, stride 1, pad 1) -- tools/conv_tune.py SHAPES
    ("3x3 64->64 256x512", 64, 64, 256, 512, 8),
    ("3x3 128->128 128x256", 128, 128, 128, 256, 8),
    ("3x3 256->256 64x128", 256, 256, 64, 128, 8),
    ("3x3 448->24 256x512", 448, 24, 256, 512, 8),
    ("3x3 256->64 256x512", 256, 64, 256, 512, 8),
    ("3x3 64->256 256x512", 64, 256, 256, 512, 8),
]

SHAPES = [(1 << 20, 448, 896), (1 << 20, 896, 448), (1 << 20, 448, 448), (1 << 20, 64, 256), (1 << 20, 256, 64)]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    for M, K, N in SHAPES:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        b = torch.randn(N, K, device=dev).to(torch.bfloat16)
        for tag, fn in (("x@w^T", lambda: torch.mm(a, b.t())), ("x@w", lambda: torch.mm(a, b.t().contiguous()))):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / iters
            print(f"mm {M}x{K} -> {N} {tag:6s}: {ms * 1e3:8.1f} us  {2 * M * K * N / ms / 1e9:7.1f} TF/s  "
                  f"{2 * (M * K + M * N) / ms / 1e6:7.1f} GB/s", flush=True)

    import torch.nn.functional as F
    for name, cin, cout, H, W, B in CONVS:
        x = torch.randn(B, cin, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, 3, 3, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        fn = lambda: F.conv2d(x, w, padding=1)  # noqa: E731
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        print(f"conv2d {name:24s} (MIOpen, NHWC bf16): {ms * 1e3:8.1f} us  "
              f"{2 * B * H * W * cout * cin * 9 / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
