"""Builds the reset-phase-timer diagnostic library (scripts/reset_stamps.py reads it): a COPY of
csrc/env_step.hip with s_memtime stamps after each phase of env_reset_kernel, written to
dgppo_fov_amd/_build/rdiag/env_step.hip and compiled with -DDGPPO_ENV_STAMPS into
dgppo_fov_amd/lib/libdgppo_hip_rdiag.so (the shipped sources stay stamp-free, so their hash does not move).
Run `make` first: every other object is the in-tree build."""
import glob
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "dgppo_fov_amd/csrc/env_step.hip")).read()
k0 = src.index("void env_reset_kernel(dgppo_env_cfg cfg, dgppo_env_reset_io io, int states_only) {")
b0 = src.index("{", k0) + 1
src = src[:b0] + """
  uint64_t rs_t = __builtin_amdgcn_s_memtime();
#define RSTAMP(k) do { if (threadIdx.x == 0) { const uint64_t now_ = __builtin_amdgcn_s_memtime(); \\
    atomicAdd(&wv::g_env_stamps[k], (unsigned long long)(now_ - rs_t)); rs_t = now_; } } while (0)
""" + src[b0:]
marks = [("  if (tid == 0) rng_count = (uint32_t)n_ob_draws;\n  __syncthreads();\n", 0),
         ("    tab[2 * k + 1] = r.uniform(0.0f, area);\n  }\n  __syncthreads();\n", 1),
         ("    if (tid == 0) rng_count = rng.count;\n  }\n  __syncthreads();\n", 2),
         ("    goal[idx] = c < 2 ? gl[2 * i + c] : 0.0f;\n  }\n  __syncthreads();\n", 3),
         ("        for (int c = 0; c < SD; ++c) third[o * SD + c] = c == 0 ? cx : (c == 1 ? cy : 0.0f);\n"
          "      }\n    }\n  }\n  __syncthreads();\n", 4),
         ("  if (states_only) {  // the wave step kernel builds the graph from these rows (dgppo_env_reset)\n", 5),
         ("    write_graph<ENGINE, GOAL, SD>(cfg, d, nxt, goal, mpe ? third : lds + cv.hits, out, vec4, tid, BLOCK);\n"
          "  }\n", 7)]
pos = b0
for anchor, k in marks:
    i = src.index(anchor, pos) + len(anchor)
    src = src[:i] + f"  RSTAMP({k});\n" + src[i:]
    pos = i
out = os.path.join(ROOT, "dgppo_fov_amd/_build/rdiag")
os.makedirs(out, exist_ok=True)
open(os.path.join(out, "env_step.hip"), "w").write(src)
hipcc = "/opt/rocm/bin/hipcc"
obj = os.path.join(ROOT, "dgppo_fov_amd/_build/env_step_rdiag.o")
subprocess.check_call([hipcc, "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-Iinclude", "-Idgppo_fov_amd/csrc",
                       "-DDGPPO_ENV_STAMPS", "-c", os.path.join(out, "env_step.hip"), "-o", obj], cwd=ROOT)
objs = [o for o in sorted(glob.glob(os.path.join(ROOT, "dgppo_fov_amd/_build/*.o"))) if "env_step" not in os.path.basename(o)]
subprocess.check_call([hipcc, "--offload-arch=gfx950", "-shared", "-o",
                       os.path.join(ROOT, "dgppo_fov_amd/lib/libdgppo_hip_rdiag.so")] + objs + [obj], cwd=ROOT)
print("built dgppo_fov_amd/lib/libdgppo_hip_rdiag.so")
