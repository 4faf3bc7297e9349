"""Time the GEMM entry point on the update's dominant shapes (scripts/gemm_shapes.py) and print the
achieved HBM rate (A + B + C bytes, C read too when beta != 0) per shape.  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.nn import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("ROWS", "131072"))
# (label, M, N, K, ta, tb, batch, bias, beta)
SHAPES = [
    ("fwd N192 K64 +b", M, 192, 64, 0, 0, 1, True, 0.0),
    ("fwd N64 K64 relu K64", M, 64, 64, 0, 0, 1, True, 0.0),
    ("fwd N64 K64 +b", M, 64, 64, 0, 0, 1, True, 0.0),
    ("dx N64 K192 tb", M, 64, 192, 0, 1, 1, False, 0.0),
    ("dx N64 K64 tb", M, 64, 64, 0, 1, 1, False, 0.0),
    ("fwd N64 K111", M, 64, 111, 0, 0, 1, False, 0.0),
    ("dx N111 K64 tb", M, 111, 64, 0, 1, 1, False, 0.0),
    ("fwd N192 K32 +b", M, 192, 32, 0, 0, 1, True, 0.0),
    ("fwd N99 K32 +b", M, 99, 32, 0, 0, 1, True, 0.0),
    ("fwd N64 K32 +b +add relu", M, 64, 32, 0, 0, 1, True, 0.0),
    ("dx N32 K192 tb", M, 32, 192, 0, 1, 1, False, 0.0),
    ("wgrad M64 N192", 64, 192, M, 1, 0, 1, False, 1.0),
    ("wgrad M64 N64", 64, 64, M, 1, 0, 1, False, 1.0),
    ("wgrad M111 N64", 111, 64, M, 1, 0, 1, False, 1.0),
    ("wgrad M32 N192", 32, 192, M, 1, 0, 1, False, 1.0),
    ("wgrad M32 N99 (Gaug)", 32, 99, M, 1, 0, 1, False, 0.0),
    ("wgrad M8 N27 (Gaug)", 8, 27, M, 1, 0, 1, False, 0.0),
]
iters = int(os.environ.get("ITERS", "20"))
if os.environ.get("COPY", "0") == "1":  # HBM calibration: read + write of an (M, 64) fp32 buffer
    X = torch.randn((M, 64), device=dev)
    Y = torch.empty_like(X)
    for _ in range(3):
        Y.copy_(X)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        Y.copy_(X)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    print(f"copy (M, 64) fp32: {us:8.1f} us  {8 * X.numel() / us / 1e3:7.0f} GB/s")
only = os.environ.get("SHAPE")  # substring filter on the label
for (lab, m, n, k, ta, tb, batch, bias, beta) in SHAPES:
    if only and only not in lab:
        continue
    A = torch.randn((k, m) if ta else (m, k), device=dev)
    B = torch.randn((n, k) if tb else (k, n), device=dev)
    C = torch.zeros((m, n), device=dev)
    bv = torch.randn(n, device=dev) if bias else None
    bg = torch.zeros(n, device=dev) if ta else None

    add = torch.randn((m, n), device=dev) if "+add" in lab else None

    def run():
        K.gemm(A, B, C, m, n, k, ta=bool(ta), tb=bool(tb), bias=bv, beta=beta, bias_grad=bg, addend=add,
               relu="relu" in lab)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    byts = 4 * (A.numel() + B.numel() + C.numel() * (2 if beta else 1))
    print(f"{lab:18s} M={m:7d} N={n:4d} K={k:7d}: {us:8.1f} us  {byts / us / 1e3:7.0f} GB/s  "
          f"{2 * m * n * k / us / 1e6:6.1f} TF/s")
