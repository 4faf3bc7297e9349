"""The oracle reproduces the committed golden fixtures bit for bit (regression pin)."""
import glob
import os

import numpy as np
import pytest

from oracle import env as O

FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "env_*.npz")))


def test_fixtures_exist():
    assert len(FILES) >= 6


@pytest.mark.parametrize("fn", FILES, ids=[os.path.basename(f) for f in FILES])
def test_oracle_reproduces_golden(fn):
    z = np.load(fn, allow_pickle=False)
    spec = O.Spec(str(z["env_id"]), int(z["n"]), int(z["n_obs"]))
    B = z["states0"].shape[0]
    ag, gl, third = O.env_reset(spec, int(z["seed"]), B)
    g0 = O.initial_graph(spec, ag, gl, third)
    np.testing.assert_array_equal(g0["states"], z["states0"])
    out = O.env_step(spec, z["states0"], z["third0"] if spec.engine != O.ENGINE_MPE else None, z["action"])
    for f in ("nodes", "edges", "states", "receivers", "senders", "reward", "cost"):
        np.testing.assert_array_equal(out[f], z[f], err_msg=f)
