"""Summarise the long learning runs (scripts/long_run.sh; gpurun_out/long/LidarSpread/<algo>/seed*/log.jsonl) into
one JSON: per run the eval curve every 50 updates (reward, cost, unsafe_frac on the 32 fixed test envs, trainer.py
:103-125) and the update diagnostics logged every 50 updates (safe_data, Vh column means on the rollout and on the
det rollout, the det-rollout Qh targets and costs, train-rollout unsafe fraction / act_drift, entropy), plus
milestones: the first update from which the eval unsafe_frac stays <= 0.1 for 10 consecutive evals, and windowed
means over the last 5000 updates.
  python scripts/long_summary.py gpurun_out/long profiles/r04_learning_long.json [ENV]"""
import glob
import json
import os
import sys

root, out_path = sys.argv[1], sys.argv[2]
ENV = sys.argv[3] if len(sys.argv) > 3 else "LidarSpread"
KEYS = ("eval/safe_data", "Vh/mean_h0", "Vh/mean_h1", "Vh/det_mean_h0", "Vh/det_mean_h1", "Vh/det_target_mean_h0",
        "Vh/det_target_mean_h1", "det/cost_mean_h0", "det/cost_mean_h1", "train/unsafe_frac", "train/act_drift",
        "train/reward", "policy/entropy", "policy/clip_frac", "Vl/loss", "Vh/loss_Vh")
runs = {}
for run in sorted(glob.glob(os.path.join(root, ENV, "*", "seed*"))):
    algo = os.path.basename(os.path.dirname(run))
    rows = [json.loads(x) for x in open(os.path.join(run, "log.jsonl"))]
    ev = [r for r in rows if "eval/reward" in r]
    up = [r for r in rows if "Vl/loss" in r]
    curve = [[r["step"], round(r["eval/reward"], 4), round(r["eval/cost"], 4), round(r["eval/unsafe_frac"], 4)] for r in ev]
    diag = [[r["step"]] + [round(float(r.get(k, float("nan"))), 4) for k in KEYS] for r in up]
    safe_from = None
    for k in range(len(curve) - 10):
        if all(c[3] <= 0.1 for c in curve[k:k + 10]):
            safe_from = curve[k][0]
            break
    last = curve[-1][0]
    tail = [c for c in curve if c[0] > last - 5000]
    mean = lambda xs: round(sum(xs) / len(xs), 4) if xs else None  # noqa: E731
    runs[f"{algo}_{os.path.basename(run).split('_')[0]}"] = {
        "algo": algo, "updates": last, "eval_every": 50, "n_env_train": 128, "n_env_test": 32,
        "first_update_eval_unsafe_le_0.1_for_10_evals": safe_from,
        "last_5000_updates": {"eval_reward": mean([c[1] for c in tail]), "eval_cost": mean([c[2] for c in tail]),
                              "eval_unsafe_frac": mean([c[3] for c in tail])},
        "eval_at_0": curve[0], "eval_curve_keys": ["update", "eval/reward", "eval/cost", "eval/unsafe_frac"],
        "eval_curve": curve, "diag_keys": ["update"] + list(KEYS), "diag_every_50": diag}
out = {"what": f"README quickstart (python train.py --env {ENV} --algo <algo> -n 3 --obs 3; reference defaults: "
               "128 envs, batch 16384, --steps 200000 CBF schedule, eval every 50 updates on 32 envs), resumed across "
               "gpurun calls (train.py --resume, bit-exact host RNG / Adam state)",
       "runs": runs}
json.dump(out, open(out_path, "w"))
for k, v in runs.items():
    print(k, v["updates"], v["first_update_eval_unsafe_le_0.1_for_10_evals"], v["last_5000_updates"], v["eval_at_0"])
