"""Probe: what the vendor GEMM (torch.mm -> hipBLASLt / rocBLAS, bf16) reaches on the
GEMM shapes of the HRNet convolutions (pixels x K) @ (K x cout), to calibrate the conv
kernels' headroom.  Prints ms and TFLOP/s (and GB/s of A + C + B)."""
import sys
import torch

dev = torch.device("cuda:0")
N = 8 * 256 * 512
shapes = [  # (pixels, K, cout, note)
    (N, 448, 448, "1x1 448->448 full"), (N, 256, 64, "1x1 256->64 full"), (N, 64, 256, "1x1 64->256 full"),
    (N, 576, 64, "3x3 64->64 full (im2col K)"), (N // 4, 1152, 128, "3x3 128->128 half"),
    (N // 16, 2304, 256, "3x3 256->256 quarter"), (N, 448 * 9, 8, "3x3 448->3 head"),
]
for M, K, Nc, note in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, Nc, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * M * K * Nc
    by = 2.0 * (M * K + M * Nc + K * Nc)
    print(f"{note:30s} M={M:8d} K={K:5d} N={Nc:4d}  {ms:7.3f} ms  {fl / ms / 1e9:7.1f} TFLOP/s  {by / ms / 1e6:7.1f} GB/s",
          flush=True)
