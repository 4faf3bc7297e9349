"""Regenerate tests/golden/env_*.npz from the NumPy oracle (oracle/env.py).

These are data fixtures (inputs + expected outputs) for small cases of every BASELINE.json
env config, plus LidarOmniTarget.  The reference itself cannot produce them (JAX absent — parity unpinned); they pin
the restatement against regressions and give the GPU tests a fixed target.
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import env as O  # noqa: E402

CASES = [("MPETarget", 3, 0, 4, 11), ("MPESpread", 3, 3, 4, 12), ("LidarSpread", 8, 3, 4, 13),
         ("LidarBicycleTarget", 8, 3, 4, 14), ("LidarSpread", 32, 8, 2, 15), ("LidarTarget", 4, 2, 4, 16),
         ("LidarOmniTarget", 8, 3, 4, 17)]


def make(eid, n, obs, B, seed):
    spec = O.Spec(eid, n, obs)
    ag, gl, third = O.env_reset(spec, seed, B)
    g0 = O.initial_graph(spec, ag, gl, third)
    a = np.random.default_rng(seed).uniform(-1, 1, (B, n, spec.ad)).astype(np.float32)
    if spec.ad == 3:
        a[..., 2] *= 1500.0  # Omni angular acceleration: part of it beyond the +-1000 clip
    out = O.env_step(spec, g0["states"], third if spec.engine != O.ENGINE_MPE else None, a)
    return dict(env_id=np.array(eid), n=np.array(n), n_obs=np.array(obs), seed=np.array(seed),
                states0=g0["states"], third0=third, action=a, nodes=out["nodes"], edges=out["edges"],
                states=out["states"], receivers=out["receivers"], senders=out["senders"],
                reward=out["reward"], cost=out["cost"])


if __name__ == "__main__":
    for c in CASES:
        d = make(*c)
        fn = os.path.join(HERE, f"env_{c[0]}_n{c[1]}_o{c[2]}.npz")
        np.savez_compressed(fn, **d)
        print(fn, os.path.getsize(fn))
