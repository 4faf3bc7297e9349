import os, sys, torch
sys.path.insert(0, "/root/repo")
from dgppo_fov_amd.nn import kernels as K
dev = torch.device("cuda:0")
M = int(os.environ.get("M", "32"))
for (n, k) in [(64, 16), (64, 64), (64, 192), (32, 64), (192, 64)]:
    A = torch.randn(M, k, device=dev); B = torch.randn(k, n, device=dev); C = torch.empty(M, n, device=dev)
    for _ in range(20):
        K.gemm(A, B, C, M, n, k)
    torch.cuda.synchronize()
    print("done", n, k, flush=True)
