"""End to end through the reference's entry points: train.py (make_env / make_algo / Trainer: collect,
update, eval, checkpoint) for a few iterations, then test.py on the saved checkpoint (deterministic
rollouts, returns / max cost / safe rate), in this process, for a Lidar env and LidarOmniTarget."""
import glob
import importlib.util
import json
import math
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def _entry(name):  # the repo-root scripts by path (`test` would also name the stdlib package)
    spec = importlib.util.spec_from_file_location(f"dgppo_entry_{name}", os.path.join(ROOT, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("eid,n,obs,algo,extra", [
    ("LidarSpread", 3, 2, "dgppo", []), ("LidarOmniTarget", 3, 2, "dgppo", []), ("LidarSpread", 3, 2, "informarl", []),
    ("LidarSpread", 3, 2, "hcbfcrpo", []),
    # the network options of the reference CLI: 2-layer LSTM, a 3-layer actor GNN; no RNN with InforMARL-Lagr
    ("LidarSpread", 3, 2, "dgppo", ["--use-lstm", "--rnn-layers", "2", "--actor-gnn-layers", "3"]),
    ("LidarSpread", 3, 2, "informarl_lagr", ["--no-rnn"])], ids=lambda v: "-".join(v) if isinstance(v, list) else None)
def test_train_then_test_entry_points(cuda, tmp_path, monkeypatch, capsys, eid, n, obs, algo, extra):
    test_py, train_py = _entry("test"), _entry("train")

    argv = ["train.py", "--env", eid, "-n", str(n), "--algo", algo, "--obs", str(obs), "--steps", "2",
            "--n-env-train", "8", "--batch-size", "256", "--n-env-test", "4", "--eval-interval", "1",
            "--save-interval", "2", "--log-dir", str(tmp_path)] + extra
    monkeypatch.setattr(sys, "argv", argv)
    train_py.main()
    runs = glob.glob(os.path.join(str(tmp_path), eid, algo, "seed0_*"))
    assert len(runs) == 1
    run = runs[0]
    assert os.path.exists(os.path.join(run, "config.yaml"))
    assert sorted(os.listdir(os.path.join(run, "models"))) == ["0", "2"]
    rows = [json.loads(x) for x in open(os.path.join(run, "log.jsonl"))]
    assert rows and all(math.isfinite(v) for r in rows for v in r.values() if isinstance(v, float))
    assert any("eval/safe_data" in r or "eval/unsafe_frac" in r for r in rows)
    capsys.readouterr()
    monkeypatch.setattr(sys, "argv", ["test.py", "--path", run, "--epi", "4", "--max-step", "16", "--no-video"])
    test_py.main()
    out = capsys.readouterr().out
    assert "safe_rate:" in out and "reward:" in out and out.count("epi: ") == 4
    # the reference's generalisation eval: more agents / obstacles than training, skip 1 episode, log a csv row
    argv = ["test.py", "--path", run, "--epi", "5", "--offset", "1", "-n", str(n + 1), "--obs", str(obs + 1),
            "--max-step", "16", "--log", "--no-video"]
    monkeypatch.setattr(sys, "argv", argv)
    test_py.main()
    out = capsys.readouterr().out
    assert out.count("epi: ") == 4 and "epi: 0," not in out and "epi: 4," in out
    row = open(os.path.join(run, "test_log.csv")).read().strip().split(",")
    assert len(row) == 7 and row[0] == str(n + 1) and row[1] == "5" and row[2] == "16" and row[4] == str(obs + 1)
    assert 0.0 <= float(row[5]) <= 100.0
