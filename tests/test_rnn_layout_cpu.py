"""Host-side carry layout of the RNN options (--rnn-layers / --use-lstm / --no-rnn): the reference's
(..., rnn_layers, n, carries, 64) carries <-> the kernels' agent-major (..., n, W) rows (DGPPO._rows / _unrows),
and the RNNStack carry widths and parameter names."""
import types

import pytest
import torch

from dgppo_fov_amd.algo.dgppo import DGPPO
from dgppo_fov_amd.nn.layers import ParamSpace, RNNStack


@pytest.mark.parametrize("layers,carries", [(1, 1), (2, 1), (1, 2), (3, 2)])
def test_carry_rows_round_trip(layers, carries):
    B, T, n = 3, 4, 5
    ref = torch.randn(B, T, layers, n, carries, 64)
    rows = DGPPO._rows(ref)
    assert rows.shape == (B, T, n, layers * carries * 64)
    # agent a's row holds its (layer, carry) blocks in order
    for lay in range(layers):
        for c in range(carries):
            off = (lay * carries + c) * 64
            assert torch.equal(rows[1, 2, 3, off:off + 64], ref[1, 2, lay, 3, c])
    fake = types.SimpleNamespace(rnn_layers=layers, n_carries=carries)
    assert torch.equal(DGPPO._unrows(fake, rows), ref)
    # the rollout engine's (T+1, B, n, W) buffer read as the reference layout is a view, and _rows undoes it
    buf = torch.randn(T + 1, B, n, layers * carries * 64)
    view = buf[:T].transpose(0, 1).unflatten(-1, (layers, carries, 64)).movedim(-4, -3)
    assert view.shape == (B, T, layers, n, carries, 64) and view.data_ptr() == buf.data_ptr()
    assert torch.equal(DGPPO._rows(view), buf[:T].transpose(0, 1))


@pytest.mark.parametrize("kind,layers,W,names", [
    ("gru", 1, 64, {"rnn.Wi", "rnn.bi", "rnn.Wh", "rnn.bhn"}),
    ("gru", 2, 128, {"rnn.GRUCell_1.Wh"}),
    ("lstm", 2, 256, {"rnn.LSTMCell_0.Wi", "rnn.LSTMCell_1.b"}),
    ("none", 3, 192, set())])
def test_rnn_stack_widths_and_params(kind, layers, W, names):
    ps = ParamSpace()
    st = RNNStack(ps, "rnn", kind, layers)
    assert st.W == W and st.layers == layers and st.carries == (2 if kind == "lstm" else 1)
    got = {n for n, _, _ in ps.entries}
    assert names <= got and (kind != "none" or not got)
    with pytest.raises(ValueError):
        RNNStack(ParamSpace(), "rnn", "lstm", 0)
