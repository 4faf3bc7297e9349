"""train.py --resume argument check: the saved world size is part of a run's identity, because it
scales the batch size and the env sharding (train.py `batch_size * world`)."""
import argparse
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import train  # noqa: E402


def _args(**kw):
    d = dict(env="LidarSpread", num_agents=3, lr_actor=3e-4, resume=None, max_minutes=None)
    d.update(kw)
    return argparse.Namespace(**d)


def test_resume_refuses_a_different_world_size(tmp_path):
    with open(tmp_path / "train_args.json", "w") as f:
        json.dump(dict(vars(_args()), _world_size=2), f)
    train.check_resume_args(_args(resume=str(tmp_path), max_minutes=5), str(tmp_path), world=2)  # resume-only flags
    with pytest.raises(SystemExit, match="_world_size"):
        train.check_resume_args(_args(resume=str(tmp_path)), str(tmp_path), world=1)
    with pytest.raises(SystemExit, match="lr_actor"):
        train.check_resume_args(_args(lr_actor=1e-4), str(tmp_path), world=2)


def test_runs_saved_without_a_world_size_count_as_one_gpu(tmp_path):
    with open(tmp_path / "train_args.json", "w") as f:
        json.dump(vars(_args()), f)
    train.check_resume_args(_args(), str(tmp_path), world=1)
    with pytest.raises(SystemExit, match="_world_size"):
        train.check_resume_args(_args(), str(tmp_path), world=8)
