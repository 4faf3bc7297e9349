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


def test_resume_continues_the_exact_sequence(cuda, tmp_path, monkeypatch):
    """a run stopped by --max-minutes after 2 updates and continued with --resume ends with the same
    parameters, Adam moments / counts and update log as the same run trained in one go (models/<k> = the state
    before update k; the final resumable state is models/<steps + 1>)."""
    import torch

    train_py = _entry("train")
    from dgppo_fov_amd.trainer import trainer as trainer_mod

    base = ["train.py", "--env", "LidarSpread", "-n", "3", "--algo", "dgppo", "--obs", "2", "--steps", "3",
            "--n-env-train", "8", "--batch-size", "256", "--n-env-test", "4", "--eval-interval", "2",
            "--save-interval", "100", "--max-minutes", "1000"]

    def run(log_dir, extra=()):
        monkeypatch.setattr(sys, "argv", base + ["--log-dir", str(log_dir)] + list(extra))
        return train_py.main()

    run(tmp_path / "once")
    calls = {"n": 0}

    def stop_at_step_2(self, start_time):  # the stop check runs once at the top of every step
        calls["n"] += 1
        return calls["n"] == 3

    with monkeypatch.context() as m:
        m.setattr(trainer_mod.Trainer, "_out_of_time", stop_at_step_2)
        run(tmp_path / "split")
    (split,) = glob.glob(os.path.join(str(tmp_path / "split"), "LidarSpread", "dgppo", "seed0_*"))
    st = json.load(open(os.path.join(split, "trainer_state.json")))
    assert st["next_step"] == 2 and sorted(os.listdir(os.path.join(split, "models"))) == ["0", "2"]
    with pytest.raises(SystemExit):  # a resume with other hyperparameters is refused
        run(tmp_path / "split", ["--resume", split, "--lr-actor", "1e-4"])
    run(tmp_path / "split", ["--resume", split])
    (once,) = glob.glob(os.path.join(str(tmp_path / "once"), "LidarSpread", "dgppo", "seed0_*"))
    for net in ("actor", "Vl", "Vh"):
        a = torch.load(os.path.join(once, "models", "4", f"{net}.pt"), weights_only=True)
        b = torch.load(os.path.join(split, "models", "4", f"{net}.pt"), weights_only=True)
        for k in ("params", "m", "v", "state"):
            assert torch.equal(a[k], b[k]), (net, k)
    strip = lambda rows: [{k: v for k, v in r.items() if not k.startswith("time")} for r in rows]  # noqa: E731
    la = strip([json.loads(x) for x in open(os.path.join(once, "log.jsonl"))])
    lb = strip([json.loads(x) for x in open(os.path.join(split, "log.jsonl"))])
    assert la == lb
