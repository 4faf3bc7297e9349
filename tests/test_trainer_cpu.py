"""Evaluation metrics of the trainer / test.py (trainer.py:103-116, test.py:103-139) on hand-built
rollouts, and the Trainer's params contract."""
import numpy as np
import pytest

from dgppo_fov_amd.trainer.trainer import Trainer
from dgppo_fov_amd.trainer.utils import eval_info, safe_rate


def test_eval_info_matches_reference_formulas():
    rng = np.random.default_rng(0)
    r = rng.standard_normal((4, 6))
    c = rng.standard_normal((4, 6, 3, 2)) * 0.1
    info = eval_info(r, c)
    assert np.isclose(info["eval/reward"], r.sum(-1).mean())
    assert np.isclose(info["eval/reward_final"], r[:, -1].mean())
    assert np.isclose(info["eval/cost"], np.maximum(c, 0).max(-1).max(-1).sum(-1).mean())
    assert np.isclose(info["eval/unsafe_frac"], (c.max(-1).max(-2) >= 1e-6).mean())


def test_safe_rate_definition():
    c = -np.ones((2, 5, 4, 2))
    c[0, 3, 1, 0] = 0.0   # env 0: agent 1 touches the constraint once -> 3/4 safe
    c[1, :, :, 1] = 0.2   # env 1: every agent unsafe
    assert np.allclose(safe_rate(c), [0.75, 0.0])


def test_trainer_params_contract():
    ok = {"run_name": "x", "training_steps": 1, "eval_interval": 1, "eval_epi": 1, "save_interval": 1}
    assert Trainer._check_params(ok)
    for k in ok:
        bad = dict(ok)
        bad.pop(k)
        with pytest.raises(AssertionError):
            Trainer._check_params(bad)
