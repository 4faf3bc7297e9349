"""A DGPPO learning run through the reference's entry points: train.py (LidarSpread n=8 obs=3, the
reference defaults: --n-env-train 128, --batch-size 16384, rnn_step 16, eval every --eval-interval
steps on 32 deterministic envs) and then test.py on the final checkpoint (--epi episodes).  Writes
the eval curve and the test summary to <out>/learning_run.json.

  python scripts/learning_run.py --steps 1000 --out gpurun_out/learn
"""
import argparse
import glob
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _entry(name):
    spec = importlib.util.spec_from_file_location(f"dgppo_entry_{name}", os.path.join(ROOT, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="LidarSpread")
    ap.add_argument("-n", type=int, default=8)
    ap.add_argument("--obs", type=int, default=3)
    ap.add_argument("--algo", default="dgppo")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--eval-interval", type=int, default=50)
    ap.add_argument("--epi", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/learn")
    a, extra = ap.parse_known_args()  # anything else goes to train.py (e.g. --lr-actor 1e-4)
    os.makedirs(a.out, exist_ok=True)
    train, test = _entry("train"), _entry("test")
    t0 = time.time()
    sys.argv = ["train.py", "--env", a.env, "-n", str(a.n), "--algo", a.algo, "--obs", str(a.obs), "--steps",
                str(a.steps), "--eval-interval", str(a.eval_interval), "--save-interval", str(a.steps),
                "--seed", str(a.seed), "--log-dir", os.path.join(a.out, "logs")] + extra
    train.main()
    t_train = time.time() - t0
    (run,) = glob.glob(os.path.join(a.out, "logs", a.env, a.algo, f"seed{a.seed}_*"))
    rows = [json.loads(x) for x in open(os.path.join(run, "log.jsonl"))]
    evals = [r for r in rows if "eval/reward" in r]
    res = {}
    for step in (0, a.steps):
        res[step] = test.test(argparse.Namespace(**{**vars(_test_args(test)), "path": run, "epi": a.epi, "step": step,
                                                    "log": True}))
    out = {"env": a.env, "n": a.n, "obs": a.obs, "algo": a.algo, "steps": a.steps, "train_args": extra,
           "env_vars": {k: v for k, v in os.environ.items() if k.startswith("DGPPO_")}, "train_wall_s": round(t_train, 1),
           "s_per_iteration": round(t_train / (a.steps + 1), 4),
           "eval_curve": [{k: r[k] for k in ("step", "eval/reward", "eval/cost", "eval/unsafe_frac")} for r in evals],
           "test_untrained_step0": res[0], f"test_step{a.steps}": res[a.steps], "test_epi": a.epi,
           "update_tail": [{k: v for k, v in r.items() if not k.startswith("eval/")} for r in rows
                           if "Vl/loss" in r][-3:],
           "update_curve": [[r["step"]] + [round(float(r.get(k, float("nan"))), 4) for k in CURVE_KEYS]
                            for r in rows if "Vl/loss" in r][::max(1, a.steps // 30)],
           "update_curve_keys": ["step"] + list(CURVE_KEYS)}
    with open(os.path.join(a.out, "learning_run.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("train_wall_s", "test_untrained_step0", f"test_step{a.steps}")}))


CURVE_KEYS = ("train/reward", "train/unsafe_frac", "train/act_drift", "eval/safe_data", "Vl/loss", "Vh/loss_Vh",
              "policy/clip_frac", "policy/entropy", "policy/total_variation_dist")


def _test_args(test):
    """test.py's argparse defaults."""
    return argparse.Namespace(path=None, no_video=True, epi=5, step=None, obs=None, stochastic=False,
                              full_observation=False, debug=False, cpu=False, max_step=None, log=False,
                              num_agents=None, seed=1234, env=None, offset=0, dpi=100)


if __name__ == "__main__":
    main()
