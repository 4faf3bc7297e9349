"""Join scripts/mfma_pmc.sh's passes: per kernel family, executed fp32 MFMA flops (SQ_INSTS_VALU_MFMA_MOPS_F32
x 512), kernel time from the un-instrumented trace, achieved TFLOP/s and the fraction of the 157.3 TFLOP/s
fp32 MFMA peak, plus MFMA busy cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs).  Only the last update_smoke
iteration (the second collect + update) is counted: kernels are grouped by dispatch order halves."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
PEAK = 157.3e12


def family(name):
    n = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(gemm_rows|gemm_wgrad_reduce|gemm_wgrad|attn_\w+?_kernel|gru_seq_\w+?_kernel|policy_step_kernel|"
                  r"lidar_step_wave_kernel|layernorm64_\w+?_kernel|gae_kernel|adam_kernel)", n)
    return m.group(1) if m else "other"


def second_half(rows, key):
    rows = sorted(rows, key=key)
    return rows[len(rows) // 2:]


pmc = defaultdict(lambda: defaultdict(float))
prow = list(csv.DictReader(open(glob.glob(os.path.join(root, "pmc", "**", "*counter_collection.csv"), recursive=True)[0])))
disp = sorted({int(r["Dispatch_Id"]) for r in prow})
keep = set(disp[len(disp) // 2:])
for r in prow:
    if int(r["Dispatch_Id"]) in keep:
        pmc[family(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
trows = list(csv.DictReader(open(glob.glob(os.path.join(root, "trace", "**", "*kernel_trace.csv"), recursive=True)[0])))
trows = second_half(trows, lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(float)
for r in trows:
    dur[family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
span = (max(int(r["End_Timestamp"]) for r in trows) - min(int(r["Start_Timestamp"]) for r in trows)) * 1e-9
out = {"peak_tflops_fp32_mfma": 157.3, "window": "second collect + update of update_smoke (LidarSpread n8, 4096 envs)",
       "window_s": round(span, 4), "families": {}}
tot_f = 0.0
for fam in sorted(set(pmc) | set(dur), key=lambda f: -dur.get(f, 0)):
    f = pmc[fam].get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) * 512
    tot_f += f
    t = dur.get(fam, 0.0)
    g = pmc[fam].get("GRBM_GUI_ACTIVE", 0.0)
    busy = pmc[fam].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    out["families"][fam] = {"time_ms": round(t * 1e3, 3), "mfma_tflop": round(f / 1e12, 4),
                            "achieved_tflops": round(f / t / 1e12, 2) if t else None,
                            "frac_of_peak": round(f / t / PEAK, 4) if t else None,
                            "mfma_busy_frac": round(busy / (g / 8 * 1024), 4) if g else None}
out["total_mfma_tflop"] = round(tot_f / 1e12, 4)
out["total_mfma_tflops_over_window"] = round(tot_f / span / 1e12, 2)
# the update alone: every dispatch after the last `spin_kernel` marker update_smoke.py launches between the
# second collect and its update (the counter pass and the trace pass run the same dispatch sequence)
marks = [r for r in trows if "spin_kernel" in r["Kernel_Name"]]
pmarks = sorted(int(r["Dispatch_Id"]) for r in prow if "spin_kernel" in r["Kernel_Name"])
if marks:
    t_mark = max(int(r["End_Timestamp"]) for r in marks)
    upd = [r for r in trows if int(r["Start_Timestamp"]) >= t_mark]
    d_mark = pmarks[-1] if pmarks else None
    uf = sum(float(r["Counter_Value"]) * 512 for r in prow if r["Counter_Name"] == "SQ_INSTS_VALU_MFMA_MOPS_F32"
             and d_mark is not None and int(r["Dispatch_Id"]) > d_mark)
    uspan = (max(int(r["End_Timestamp"]) for r in upd) - min(int(r["Start_Timestamp"]) for r in upd)) * 1e-9
    out["update_window_s"] = round(uspan, 4)
    out["update_mfma_tflop"] = round(uf / 1e12, 4)
    out["update_executed_tflops"] = round(uf / uspan / 1e12, 2)
    out["update_frac_of_peak"] = round(uf / uspan / PEAK, 4)
# VALU fp32 flops (SQ_INSTS_VALU_FLOPS_FP32 + _TRANS), calibrated on the known elementwise work of valu_calib.py
# (torch.mul: 1 flop per element, torch.addcmul: 2), so `counter / per_flop` = executed fp32 VALU flops
cal = glob.glob(os.path.join(root, "calib", "**", "*counter_collection.csv"), recursive=True)
per_flop = None
if cal:
    crow = list(csv.DictReader(open(cal[0])))
    got = defaultdict(float)
    for r in crow:
        if r["Counter_Name"] == "SQ_INSTS_VALU_FLOPS_FP32":
            k = "mul" if "MulFunctor" in r["Kernel_Name"] else ("addcmul" if "addcmul" in r["Kernel_Name"] else None)
            if k:
                got[k] += float(r["Counter_Value"])
    n_el = float(1 << 24) * 2  # two launches each
    if got.get("mul"):
        per_flop = got["mul"] / n_el
        out["valu_calibration"] = {"mul_counter_per_element": round(got["mul"] / n_el, 4),
                                   "addcmul_counter_per_element": round(got.get("addcmul", 0.0) / n_el, 4),
                                   "counter_per_flop": round(per_flop, 4)}
if marks and per_flop:
    vf = sum(float(r["Counter_Value"]) for r in prow if r["Counter_Name"] in
             ("SQ_INSTS_VALU_FLOPS_FP32", "SQ_INSTS_VALU_FLOPS_FP32_TRANS") and d_mark is not None
             and int(r["Dispatch_Id"]) > d_mark) / per_flop
    out["update_valu_fp32_tflop"] = round(vf / 1e12, 4)
    out["update_executed_fp32_tflop"] = round((uf + vf) / 1e12, 4)
    out["update_executed_fp32_frac_of_peak"] = round((uf + vf) / uspan / PEAK, 4)
for fam in out["families"]:
    v = pmc[fam].get("SQ_INSTS_VALU_FLOPS_FP32", 0.0) + pmc[fam].get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0)
    if per_flop and v:
        out["families"][fam]["valu_fp32_tflop"] = round(v / per_flop / 1e12, 4)
# the build the profile measured: bench.py quotes the executed-MFMA figure only for the same sources (a hash of
# dgppo_fov_amd/csrc/* and include/dgppo_hip.h -- a rebuild of the same sources is the same build)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_sha256  # noqa: E402

out["src_sha256"] = source_sha256()
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(root, "mfma_util.json"), "w"), indent=1)
