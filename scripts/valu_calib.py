"""Calibration dispatches for the VALU flop counter (scripts/mfma_pmc.sh): known fp32 work on 2^24 elements --
x * y (one v_mul_f32 per element: 2^24 flops), torch.addcmul x + y * z (one fma: 2 flops per element) -- so the
profile can state what SQ_INSTS_VALU_FLOPS_FP32 counts per element op on gfx950."""
import torch

n = 1 << 24
x, y, z = (torch.rand(n, device="cuda") for _ in range(3))
for _ in range(2):
    torch.mul(x, y)
    torch.addcmul(x, y, z)
torch.cuda.synchronize()
