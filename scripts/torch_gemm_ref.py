"""Reference timing: torch.matmul (rocBLAS / hipBLASLt fp32) on the update's dominant GEMM shapes, to
calibrate the in-house kernels (scripts/gemm_bench.py).  Not used by the product path."""
import torch

dev = torch.device("cuda:0")
torch.backends.cuda.matmul.allow_tf32 = False
M = 131072
for (lab, m, n, k, ta) in [("N64 K64", M, 64, 64, 0), ("N192 K64", M, 192, 64, 0), ("N64 K192", M, 64, 192, 0),
                           ("N64 K111", M, 64, 111, 0), ("wgrad 64x192", 64, 192, M, 1), ("wgrad 64x64", 64, 64, M, 1)]:
    A = torch.randn((k, m) if ta else (m, k), device=dev)
    B = torch.randn((k, n), device=dev)
    f = (lambda: A.t() @ B) if ta else (lambda: A @ B)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    byts = 4 * (m * k + k * n + m * n)
    print(f"torch {lab:14s}: {us:7.1f} us  {byts / us / 1e3:6.0f} GB/s  {2 * m * n * k / us / 1e6:6.1f} TF/s")
