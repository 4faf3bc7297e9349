"""Collect gpurun_out/abl_<name>/learning_run.json files into one committed profile (eval curve, test.py
summaries and the per-update curve of each run).  python scripts/collect_ablation.py OUT.json NOTE abl_a abl_b ..."""
import json
import os
import sys

out, note, names = sys.argv[1], sys.argv[2], sys.argv[3:]
runs = {}
for name in names:
    fn = os.path.join("gpurun_out", name, "learning_run.json")
    d = json.load(open(fn))
    tk = [k for k in d if k.startswith("test_step") and k != "test_step0"][0]
    runs[name] = {"env": d["env"], "n": d["n"], "obs": d["obs"], "algo": d["algo"], "steps": d["steps"],
                  "train_args": d["train_args"], "env_vars": d.get("env_vars"),
                  "eval_curve": [[e["step"], round(e["eval/reward"], 4), round(e["eval/cost"], 3),
                                  round(e["eval/unsafe_frac"], 3)] for e in d["eval_curve"]],
                  "test_step0": d["test_untrained_step0"], "test_final": d[tk],
                  "update_curve_keys": d["update_curve_keys"], "update_curve": d["update_curve"]}
json.dump({"note": note, "eval_curve_keys": ["step", "eval/reward", "eval/cost", "eval/unsafe_frac"], "runs": runs},
          open(out, "w"), indent=1)
print(out, len(runs))
