"""Weight-gradient GEMM path (dgppo_gemm with trans_a: C = alpha A^T B + beta C, bias_grad = colsum B) against a
float64 torch reference on the update's shapes (row chunks reduced in fixed order), repeated calls bit-identical, and
the two-stage pipelined loop (DGPPO_WGRAD_PIPE=1, the default) bit-identical to the single-stage loop (=0, run in a
child process: the knob is read once per process)."""
import os
import subprocess
import sys

import pytest
import torch

from dgppo_fov_amd.nn import kernels as K

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

# (M, N, rows, grouped A rows, beta)
SHAPES = [(64, 192, 131072, 0, 1.0), (64, 64, 16384, 0, 1.0), (111, 64, 4096, 0, 0.0), (32, 99, 1000, 0, 0.0),
          (8, 27, 777, 0, 1.0), (64, 192, 20000, 7, 1.0), (128, 128, 3000, 0, 1.0), (3, 5, 2, 0, 0.0)]


def _case(dev, M, N, R, grp, beta, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    lda = M + 3 if grp else M
    if grp:  # rows grouped: grp rows of every block of grp + 2 rows (a_gstride), the rest skipped
        nb = (R + grp - 1) // grp
        A = torch.randn((nb * (grp + 2), lda), device=dev, generator=g)
        idx = torch.cat([torch.arange(b * (grp + 2), b * (grp + 2) + grp, device=dev) for b in range(nb)])[:R]
        Ad = A[idx, :M]
    else:
        A = torch.randn((R, lda), device=dev, generator=g)
        Ad = A[:, :M]
    B = torch.randn((R, N), device=dev, generator=g)
    C = torch.randn((M, N), device=dev, generator=g)
    bg = torch.randn(N, device=dev, generator=g)
    ref = 0.5 * (Ad.double().T @ B.double()) + beta * C.double()
    refb = 0.5 * B.double().sum(0) + beta * bg.double()
    kw = dict(a_grp=grp, a_gs=(grp + 2) * lda) if grp else {}
    K.gemm(A, B, C, M, N, R, ta=True, lda=lda, alpha=0.5, beta=beta, bias_grad=bg, **kw)
    return C, bg, ref, refb


def _results(dev):
    out = []
    for k, (M, N, R, grp, beta) in enumerate(SHAPES):
        C, bg, ref, refb = _case(dev, M, N, R, grp, beta, 11 + k)
        out.append((C.cpu(), bg.cpu(), ref.cpu(), refb.cpu()))
    torch.cuda.synchronize()
    return out


def _check(results):
    for (M, N, R, grp, beta), (C, bg, ref, refb) in zip(SHAPES, results):
        tol = 2e-6 * (R ** 0.5) * 2 + 1e-5
        assert (C.double() - ref).abs().max().item() <= tol * max(1.0, ref.abs().max().item()), (M, N, R)
        assert (bg.double() - refb).abs().max().item() <= tol * max(1.0, refb.abs().max().item()), (M, N, R)


def test_wgrad_matches_float64(cuda):
    first = _results(cuda)
    _check(first)
    for _ in range(2):  # deterministic: fixed-order chunk sums
        again = _results(cuda)
        for s, a, b in zip(SHAPES, first, again):
            assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), s


def _child(tmp_path, name, **env):
    code = (f"import sys, torch; sys.path.insert(0, {os.path.dirname(HERE)!r}); sys.path.insert(0, {HERE!r}); "
            "import test_gemm_wgrad_gpu as T; r = T._results(torch.device('cuda', 0)); "
            f"torch.save(r, {str(tmp_path / name)!r})")
    subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env), check=True, timeout=120)
    return torch.load(tmp_path / name, weights_only=True)


def test_wgrad_pipelined_loop_bit_identical(cuda, tmp_path):
    mine = _results(cuda)
    other = _child(tmp_path, "p0.pt", DGPPO_WGRAD_PIPE="0")
    for s, a, b in zip(SHAPES, mine, other):
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), s


def test_grouped_wgrad_bit_identical_to_single_launches(cuda):
    """dgppo_gemm_wgrad_grouped (K.defer_wgrad): the SHAPES problems in one grouped launch (batched entries, grouped
    rows, bias gradients, beta 0 / 1) equal their single dgppo_gemm calls bit for bit."""
    single = _results(cuda)
    class everything:  # a "gradient buffer" spanning the address space
        data_ptr = staticmethod(lambda: 0)
        numel = staticmethod(lambda: 1 << 60)

    with K.defer_wgrad(cuda, everything):
        cases = [_case(cuda, M, N, R, grp, beta, 11 + k) for k, (M, N, R, grp, beta) in enumerate(SHAPES)]
        assert len(K._DEFER[K._lib.stream_handle(cuda)]) == len(SHAPES)
    torch.cuda.synchronize()
    for s, a, (C, bg, _, _) in zip(SHAPES, single, cases):
        assert torch.equal(a[0], C.cpu()) and torch.equal(a[1], bg.cpu()), s
    # batched problems (batch = 3, strided C) through both paths
    g = torch.Generator(device=cuda).manual_seed(5)
    A = torch.randn((3, 5000, 40), device=cuda, generator=g)
    B = torch.randn((3, 5000, 70), device=cuda, generator=g)
    C0 = torch.randn((3, 40, 70), device=cuda, generator=g)
    C1 = C0.clone()
    K.gemm(A, B, C0, 40, 70, 5000, ta=True, batch=3, sa=5000 * 40, sb=5000 * 70, sc=40 * 70, beta=1.0)
    with K.defer_wgrad(cuda, C1):
        K.gemm(A, B, C1, 40, 70, 5000, ta=True, batch=3, sa=5000 * 40, sb=5000 * 70, sc=40 * 70, beta=1.0)
        assert len(K._DEFER[K._lib.stream_handle(cuda)]) == 1
    assert torch.equal(C0, C1)
