"""Phase timing of the fused policy step kernel (csrc/policy.hip built with -DPOLICY_PROBE).

`python scripts/policy_probe.py --build` (here, no GPU) compiles scripts/_probe/libpolicy_probe.so;
`python scripts/policy_probe.py` (GPU box) runs one bench-sized step (LidarSpread n=8, 4096 envs) and
prints the mean duration of every phase over the workgroups (s_memrealtime, 100 MHz) plus the
kernel time.  Outputs are garbage in probe builds (h_out holds the stamps)."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "scripts", "_probe", "libpolicy_probe.so")
PHASES = ["stage", "l0 Q/QT/beta", "l0 attention", "l0 out", "l1 Q/QT/beta", "l1 attention", "l1 out",
          "MLP head", "GRU", "ScaleHid", "mean/std/sample"]
STAMPS = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11]

if "--build" in sys.argv:
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
                           "-DPOLICY_PROBE", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "dgppo_fov_amd", "csrc", "policy.hip"), "-o", SO])
    print("built", SO)
    sys.exit(0)

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.algo.module.nets import ActorNet  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn import kernels as K  # noqa: E402
from dgppo_fov_amd.nn.layers import GraphBatch  # noqa: E402

n, B = int(os.environ.get("N_AGENTS", "8")), int(os.environ.get("N_ENV", "4096"))
dev = torch.device("cuda:0")
env = make_env(os.environ.get("ENV_ID", "LidarSpread"), n, num_obs=3, device=dev)
g = env.reset(key=0, n_env=B)
gb = GraphBatch(g.nodes, g.edges, g.receivers, g.senders, n, env.agent_candidates(dev))
net = ActorNet(env.node_dim, n, dev, seed=1)
rows = B * n
h = torch.zeros((rows, 64), device=dev)
h_out = torch.zeros((rows, 64), device=dev)
act = torch.empty((rows, 2), device=dev)
lp = torch.empty(rows, device=dev)
noise = torch.randn((rows, 2), device=dev)
fa = net._fused_args(gb)
assert fa is not None
fa.G, fa.mode = gb.G, 1
fa.cand, fa.receivers, fa.senders = K._p(gb.cand), K._p(gb.receivers), K._p(gb.senders)
fa.nodes, fa.nodes_gstride = K._p(gb.nodes), gb.N * gb.nodes.shape[2]
fa.edges, fa.edges_gstride, fa.idx_gstride = K._p(gb.edges), gb.E * 4, gb.E
fa.h_in, fa.h_out, fa.noise, fa.action, fa.log_pi = K._p(h), K._p(h_out), K._p(noise), K._p(act), K._p(lp)
probe = ctypes.CDLL(SO)
probe.dgppo_policy_step.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
probe.dgppo_policy_prepare.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
stream = _lib.stream_handle(dev)
assert probe.dgppo_policy_prepare(ctypes.byref(fa), stream) == 0
for _ in range(3):
    assert probe.dgppo_policy_step(ctypes.byref(fa), stream) == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
assert probe.dgppo_policy_step(ctypes.byref(fa), stream) == 0
e1.record()
torch.cuda.synchronize()
gpg = 16 // n  # kRowsG in csrc/policy.hip
grid = (B + gpg - 1) // gpg
st = h_out.view(torch.int64).view(-1)[: grid * 32].view(grid, 32).cpu().numpy().astype(np.float64)
sub = st[:, [12, 13, 14, 16, 17, 18]]
st = st[:, :12]
d = np.diff(st, axis=1) * 10.0 / 1e3  # 100 MHz ticks -> us
print(f"kernel {e0.elapsed_time(e1) * 1e3:.1f} us, grid {grid}, span of stamps "
      f"{(st[:, -1].max() - st[:, 0].min()) * 10 / 1e3:.1f} us, per-WG mean {(st[:, -1] - st[:, 0]).mean() * 10 / 1e3:.1f} us")
for i, name in enumerate(PHASES):
    print(f"  {name:16s} mean {d[:, i].mean():7.2f} us  p90 {np.percentile(d[:, i], 90):7.2f} us")
if (sub > 0).all():
    t = np.concatenate([st[:, 5:6], sub], 1)
    dd = np.diff(t, axis=1) * 10.0 / 1e3
    names = ["sr0 x/pre", "sr0 logits", "sr0 wsum", "sr1 x/pre", "sr1 logits", "sr1 wsum"]
    for i, nm in enumerate(names):
        print(f"    l1 {nm:16s} mean {dd[:, i].mean():7.2f} us")
