"""The GRU sequence kernels' two B-operand forms (csrc/gru.hip, ABI 10 dgppo_gru_set_form): Wh as per-lane register
MFMA fragments (default) and Wh staged in LDS (the round-3 kernels) feed the same operands to the same MFMAs in the
same order, so every output -- hs, hT, dgi, dgh, dh0 and the bhn partials -- must agree bit for bit, for one-step
(Vh) and rnn_step-long sequences and a ragged last row block.  The values themselves are checked against the
float64 oracle by tests/test_nets_gpu.py."""
import pytest
import torch

from dgppo_fov_amd import _lib
from dgppo_fov_amd.nn import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Q,L,n", [(8 * 37, 1, 8), (8 * 25, 16, 8), (3 * 11, 5, 3)])
def test_gru_register_and_lds_forms_bit_identical(cuda, Q, L, n):
    g = torch.Generator().manual_seed(Q + L)
    S = Q // n
    gi = (torch.randn(S * L * n, 192, generator=g) * 0.5).to(cuda)
    Wh = (torch.randn(64, 192, generator=g) / 8).to(cuda)
    bhn = (torch.randn(64, generator=g) * 0.1).to(cuda)
    h0 = torch.randn(Q, 64, generator=g).to(cuda)
    dhs = torch.randn(S * L * n, 64, generator=g).to(cuda)
    nblk = K.gru_seq_blocks(Q)
    outs = []
    lib = _lib.load()
    try:
        for form in (1, 0):
            assert lib.dgppo_gru_set_form(form) == 0
            hs = torch.empty(S * L * n, 64, device=cuda)
            hT = torch.empty(Q, 64, device=cuda)
            K.gru_seq(True, Q, L, n, gi, Wh, bhn, h0, hs, hT=hT)
            dgi = torch.empty(S * L * n, 192, device=cuda)
            dgh = torch.empty(S * L * n, 192, device=cuda)
            dh0 = torch.empty(Q, 64, device=cuda)
            part = torch.empty(nblk, 64, device=cuda)
            K.gru_seq(False, Q, L, n, gi, Wh, bhn, h0, hs, dhs=dhs, dgi=dgi, dgh=dgh, dh0=dh0, dbhn_part=part)
            torch.cuda.synchronize()
            outs.append((hs.cpu(), hT.cpu(), dgi.cpu(), dgh.cpu(), dh0.cpu(), part.cpu()))
    finally:
        lib.dgppo_gru_set_form(1)
    for a, b, what in zip(outs[0], outs[1], ("hs", "hT", "dgi", "dgh", "dh0", "dbhn_part")):
        assert torch.equal(a, b), what
    assert torch.isfinite(outs[0][0]).all() and outs[0][0].abs().max() > 0
