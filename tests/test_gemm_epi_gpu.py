"""The row-GEMM epilogues of ABI 9 (csrc/gemm.hip, dgppo_gemm_args.epi) against float64 references of the elementwise
passes they replace, on every row path (whole-unit prefetch K <= 32, B-in-registers K = 64, plain rows with vector and
scalar A loads; K = 2 / 7 are the tiny-K shapes of the action and raw-row layers): the ReLU backward (epi 1),
LayerNorm(64) + ReLU forward (epi 2, flax LayerNorm eps 1e-6 then relu, dgppo/nn/mlp.py:20-30) and its backward (epi 3, dscale / dbias accumulated).  Tolerances: fp32 GEMM + epilogue vs
float64, 1e-5 relative to the tensor scale (2e-5 for the backward's row reductions)."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.nn import kernels as K

pytestmark = pytest.mark.gpu


def _ln_ref(h, sc, bi):
    mean = h.mean(-1, keepdims=True)
    var = np.clip((h * h).mean(-1, keepdims=True) - mean * mean, 0, None)
    rstd = 1.0 / np.sqrt(var + 1e-6)
    pre = (h - mean) * rstd * sc + bi
    return np.maximum(pre, 0), pre, mean[:, 0], rstd[:, 0]


@pytest.mark.parametrize("M,Kd", [(1000, 32), (1000, 64), (777, 192), (70, 99), (33, 64)])
def test_layernorm_epilogues(cuda, M, Kd):
    rng = np.random.default_rng(M + Kd)
    X = rng.standard_normal((M, Kd)).astype(np.float32)
    W = (rng.standard_normal((Kd, 64)) / np.sqrt(Kd)).astype(np.float32)
    b = rng.standard_normal(64).astype(np.float32) * 0.1
    sc = (1 + 0.3 * rng.standard_normal(64)).astype(np.float32)
    bi = (0.2 * rng.standard_normal(64)).astype(np.float32)
    d = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
    y, h = torch.empty((M, 64), device=cuda), torch.empty((M, 64), device=cuda)
    mean, rstd = torch.empty(M, device=cuda), torch.empty(M, device=cuda)
    scd, bid = d(sc), d(bi)
    K.gemm(d(X), d(W), y, M, 64, Kd, bias=d(b), ln=dict(mode="fwd", scale=scd, bias=bid, h=h, mean=mean, rstd=rstd))
    torch.cuda.synchronize()
    h64 = X.astype(np.float64) @ W.astype(np.float64) + b
    y64, pre64, m64, r64 = _ln_ref(h64, sc, bi)
    assert np.abs(h.cpu().numpy() - h64).max() <= 1e-5 * np.abs(h64).max()
    assert np.abs(mean.cpu().numpy() - m64).max() <= 1e-5 * np.abs(h64).max()
    assert np.abs(rstd.cpu().numpy() - r64).max() <= 1e-4 * np.abs(r64).max()
    amb = np.abs(pre64) < 1e-4  # ReLU gates fp32 may decide either way
    err = np.abs(y.cpu().numpy() - y64)
    assert err[~amb].max() <= 1e-5 * np.abs(y64).max()
    # backward: the GEMM result dy = G Wg^T (an upstream layer's input gradient), epilogue -> dx, dscale, dbias
    Kg = 128
    G = rng.standard_normal((M, Kg)).astype(np.float32)
    Wg = (rng.standard_normal((64, Kg)) / np.sqrt(Kg)).astype(np.float32)
    ds0, db0 = rng.standard_normal(64).astype(np.float32), rng.standard_normal(64).astype(np.float32)
    dx = torch.empty((M, 64), device=cuda)
    dsd, dbd = d(ds0.copy()), d(db0.copy())
    K.gemm(d(G), d(Wg), dx, M, 64, Kg, tb=True, ldb=Kg, ln=dict(mode="bwd", scale=scd, bias=bid, h=h, mean=mean, rstd=rstd, dscale=dsd, dbias=dbd))
    torch.cuda.synchronize()
    h32 = h.cpu().numpy().astype(np.float64)  # the kernel's own h (the gates follow the fp32 forward)
    y32, pre32, m32, r32 = _ln_ref(h32, sc, bi)
    dy = G.astype(np.float64) @ Wg.astype(np.float64).T
    g = np.where(pre32 > 0, dy, 0.0)
    xh = (h32 - m32[:, None]) * r32[:, None]
    gx = g * sc
    dx64 = r32[:, None] * (gx - gx.mean(-1, keepdims=True) - xh * (gx * xh).mean(-1, keepdims=True))
    rows_ok = ~(np.abs(pre32) < 1e-5).any(-1)
    e = np.abs(dx.cpu().numpy() - dx64)[rows_ok]
    assert e.max() <= 2e-5 * np.abs(dx64).max(), e.max()
    # column sums: entries whose gate is within fp32 rounding of 0 may be counted either way
    amb = np.abs(pre32) < 1e-5
    slack_s = np.abs(dy * xh * amb).sum(0)
    slack_b = np.abs(dy * amb).sum(0)
    assert (np.abs(dsd.cpu().numpy() - (ds0 + (g * xh).sum(0))) <= 1e-4 * np.sqrt(M) + slack_s).all()
    assert (np.abs(dbd.cpu().numpy() - (db0 + g.sum(0))) <= 1e-4 * np.sqrt(M) + slack_b).all()
    # the backward's ReLU gates are the forward's, bit for bit: with dy = 1 everywhere (G = ones, Wg = I) dbias
    # counts the open gates per column, an exact integer in fp32, equal to the forward's (y > 0) count
    dbd = torch.zeros(64, device=cuda)
    K.gemm(torch.ones((M, 64), device=cuda), torch.eye(64, device=cuda), dx, M, 64, 64, tb=True, ldb=64,
           ln=dict(mode="bwd", scale=scd, bias=bid, h=h, mean=mean, rstd=rstd, dscale=torch.zeros(64, device=cuda),
                   dbias=dbd))
    torch.cuda.synchronize()
    assert torch.equal(dbd.cpu(), (y > 0).float().sum(0).cpu())


@pytest.mark.parametrize("M,N,Kd,beta", [(1000, 64, 64, 0.0), (1000, 32, 99, 1.0), (500, 64, 32, 0.0), (300, 32, 192, 1.0),
                                         (1000, 64, 2, 1.0), (777, 24, 7, 0.0)])
def test_relu_mask_epilogue(cuda, M, N, Kd, beta):
    rng = np.random.default_rng(7 + M + N)
    A = rng.standard_normal((M, Kd)).astype(np.float32)
    B = rng.standard_normal((N, Kd)).astype(np.float32)  # op(B) = B^T (the dx GEMMs' transposed weights)
    C0 = rng.standard_normal((M, N)).astype(np.float32)
    Y = np.maximum(rng.standard_normal((M, N)), 0).astype(np.float32)  # a ReLU output: ~half zeros
    C = torch.from_numpy(C0).to(cuda)
    K.gemm(torch.from_numpy(A).to(cuda), torch.from_numpy(B).to(cuda), C, M, N, Kd, tb=True, ldb=Kd, beta=beta,
           mask=torch.from_numpy(Y).to(cuda))
    torch.cuda.synchronize()
    ref = np.where(Y > 0, A.astype(np.float64) @ B.astype(np.float64).T + beta * C0, 0.0)
    assert np.abs(C.cpu().numpy() - ref).max() <= 1e-5 * np.abs(ref).max()
    assert (C.cpu().numpy()[Y == 0] == 0).all()
