"""Record every GEMM launched by one DGPPO collect + update and print shapes ranked by flops."""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn import kernels as K  # noqa: E402

n, obs, B, T = 8, 3, int(os.environ.get("N_ENV", "4096")), 128
dev = torch.device("cuda:0")
env = make_env("LidarSpread", n, num_obs=obs, max_step=T, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=16384, device=dev, train_steps=100)
r = algo.collect(algo.params, 0, n_env=B)
algo.update(r, 0)  # warm (captures the det engine)
K.GEMM_LOG = []
algo.update(r, 1)
torch.cuda.synchronize()
agg = collections.defaultdict(lambda: [0, 0.0])
for (M, N, Kd, b, ta, tb, sk, bias) in K.GEMM_LOG:
    a = agg[(M, N, Kd, b, ta, tb, sk, bias)]
    a[0] += 1
    a[1] += 2.0 * M * N * Kd * b
tot = sum(v[1] for v in agg.values())
print(f"{len(K.GEMM_LOG)} launches, {tot/1e12:.2f} TFLOP")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
    print(f"{v[1]/1e12:7.3f} TF {100*v[1]/tot:5.1f}% n={v[0]:5d}  M={k[0]} N={k[1]} K={k[2]} batch={k[3]} ta={k[4]} tb={k[5]} split={k[6]} bias={k[7]}")
