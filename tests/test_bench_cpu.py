"""bench.py's multi-rank launcher and argument checks (CPU only: the launched ranks stop before any GPU
use via the hidden --print-rank-env flag)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                             "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_gpus_n_launches_n_ranks():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--print-rank-env"], env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(int(r["RANK"]) for r in rows) == [0, 1, 2]
    assert all(r["WORLD_SIZE"] == "3" and r["LOCAL_RANK"] == r["RANK"] and r["MASTER_ADDR"] == "127.0.0.1"
               for r in rows)
    assert len({r["MASTER_PORT"] for r in rows}) == 1


def test_gpus_mismatch_with_world_size_is_refused():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--print-rank-env"], env=_env(WORLD_SIZE="4"),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=4" in out.stderr


def test_default_is_one_rank_without_launch():
    out = subprocess.run([sys.executable, BENCH, "--print-rank-env"], env=_env(), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    rows = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(rows) == 1 and rows[0]["RANK"] is None and rows[0]["WORLD_SIZE"] is None


def test_failing_rank_fails_the_launch():
    # --strong with 3 ranks: 4096 envs do not split -> every rank exits non-zero, so does the launcher
    out = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--strong", "--no-cpu-baseline"], env=_env(),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "do not split" in out.stderr
