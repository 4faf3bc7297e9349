"""Diagnostic for tests/test_update_dynamics_gpu.py::test_trajectory_matches_oracle_loop[LidarSpread-3-2]: update 0,
minibatch 0.  Prints the GPU actor gradient of gnn[0]/Dense_4/kernel column 1 beside the float64 oracle's, the
oracle re-evaluated with the TanhNormal clip threshold at its fp32 value, and the per-sample |action| range near the
threshold.  GPU only; test infrastructure (imports oracle/)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import nets_t as R  # noqa: E402
from test_update_dynamics_gpu import _algo, _trees_at  # noqa: E402
from test_update_gpu import _host, _net_trees  # noqa: E402

cuda = torch.device("cuda:0")
B, T, L = 8, 32, 16
n = 3
algo, env = _algo(cuda, "LidarSpread", n, 2, T, batch=2 * T, L=L)
nets = (("Vl", algo.Vl), ("Vh", algo.Vh), ("policy", algo.actor))
roll = algo.collect(algo.params, 100, n_env=B)
start = {k: net.ps.flat.clone() for k, net in nets}
algo.trace = {}
algo.update(roll, 0)
torch.cuda.synchronize()
tr = algo.trace
hr, hd = _host(roll, n), _host(tr["det"], n)
Ql, Qh_det, A = (tr[k].double().cpu().numpy() for k in ("Ql", "Qh_det", "A"))
mb = tr["mb"][0]
pa, pl, ph = _trees_at(algo, mb["before"])
keep = algo.grad_flat.clone()
algo.grad_flat.copy_(mb["grad"])
gpu = _net_trees(algo, grad=True)
algo.grad_flat.copy_(keep)
g_gpu = np.asarray(gpu[0]["gnn"][0]["Dense_4"]["kernel"], np.float64)
envs = np.asarray(mb["envs"])
acts = np.asarray(hr["actions"])[envs].reshape(-1)
print("envs", envs, "|a| max", np.abs(acts).max(), "n(|a| > 0.998)", int((np.abs(acts) > 0.998).sum()),
      "n(|a| >= 0.999)", int((np.abs(acts) >= 0.999).sum()))
near = np.abs(acts)[np.abs(acts) > 0.998]
print("near-threshold |a|:", np.sort(near)[-10:].tolist())


def oracle(thresh, gate=None):
    R.THRESH = thresh
    R.GATE_MODE = gate
    try:
        ts = [R.to_t(x, requires_grad=True) for x in (pa, pl, ph)]
        R.dgppo_minibatch_grads(*ts, hr, hd, envs, Ql, Qh_det, A, n, L, algo.entropy_eps.cpu().numpy(), algo.clip_eps,
                                algo.coef_ent)
        return np.asarray(R.grads(ts[0])["gnn"][0]["Dense_4"]["kernel"], np.float64)
    finally:
        R.THRESH = 0.999
        R.GATE_MODE = None


ref = oracle(0.999)
gon, goff = oracle(0.999, "on"), oracle(0.999, "off")
print("gate floor (on vs off) at col 1:", np.abs(gon - goff)[:, 1], " max", np.abs(gon - goff).max())
ref32 = oracle(float(np.float32(0.999)))
np.set_printoptions(precision=7, linewidth=200)
print("gpu   col1", g_gpu[:, 1])
print("ref   col1", ref[:, 1])
print("ref32thr  ", ref32[:, 1])
print("max |gpu - ref| per column", np.abs(g_gpu - ref).max(0))
print("max |gpu - ref32thr|", np.abs(g_gpu - ref32).max(), " max |gpu - ref|", np.abs(g_gpu - ref).max())

# ---- LN_0 input statistics per (graph, agent) row: nearly constant rows (var << eps) amplify rounding noise by
# rstd ~ 1/sqrt(eps) and their ReLU(LN) gates are decided by it
with torch.no_grad():
    pa_t = R.to_t(pa)
    gh = R._flat(hr["graph"], envs)
    z = R.gnn(pa_t["gnn"], gh, n).reshape(-1, 64)
    x0 = R.dense(z, pa_t["head"]["Dense_0"])
    var = (x0 * x0).mean(-1) - x0.mean(-1) ** 2
    zmax = z.abs().max(-1).values
    order = torch.argsort(var)[:8]
    print("rows", z.shape[0], "LN_0 input var: min", float(var.min()), "median", float(var.median()))
    for r in order.tolist():
        print(f"   row {r} (graph {r // n}, agent {r % n}) var {float(var[r]):.3e} max|gnn out| {float(zmax[r]):.3e} "
              f"n(gnn out > 0) {int((z[r] > 0).sum())}")
# ---- is the discrepancy shaped like one loss term's gradient?  the oracle without the entropy term, and the
# actor's whole gradient (every leaf) compared by direction
def oracle_all(coef_ent):
    ts = [R.to_t(x, requires_grad=True) for x in (pa, pl, ph)]
    R.dgppo_minibatch_grads(*ts, hr, hd, envs, Ql, Qh_det, A, n, L, algo.entropy_eps.cpu().numpy(), algo.clip_eps,
                            coef_ent)
    from test_update_gpu import _walk
    return {p: np.asarray(v, np.float64) for p, v, _ in _walk(R.grads(ts[0]), R.grads(ts[0]))}


from test_update_gpu import _walk  # noqa: E402
gg = {p: np.asarray(v, np.float64) for p, v, _ in _walk(gpu[0], gpu[0])}
full, noent = oracle_all(algo.coef_ent), oracle_all(0.0)
dv = np.concatenate([(gg[k] - full[k]).ravel() for k in full])
ev = np.concatenate([(noent[k] - full[k]).ravel() for k in full])
print("coef_ent", algo.coef_ent, "|gpu - ref|", np.abs(dv).max(), "|entropy grad|", np.abs(ev).max(),
      "cos(gpu - ref, -entropy grad)", float(dv @ ev / (np.linalg.norm(dv) * np.linalg.norm(ev) + 1e-30)),
      "best scale", float(dv @ ev / (ev @ ev + 1e-30)))
for k in full:
    e = np.abs(gg[k] - full[k]).max()
    print(f"   {k:40s} max|ref| {np.abs(full[k]).max():.3e} max err {e:.3e} rel {e / (np.abs(full[k]).max() + 1e-30):.2e}")
sys.exit(0)

# ---- forward comparison on the minibatch graphs: the actor trunk (GNN + MLP head) per (graph, agent) row
algo.actor.ps.flat.copy_(mb["before"]["policy"])
envs_t = torch.as_tensor(envs, device=cuda)
rg = roll.graph
nodes, edges, recv, send = algo._gather(envs_t, rg.nodes, rg.edges, rg.receivers, rg.senders)
g = algo._graph_batch(nodes, edges, recv, send).prepare()
y_gpu, _ = algo.actor._trunk(g)
y_gpu = y_gpu.double().cpu().numpy()
gh = R._flat(hr["graph"], envs)
with torch.no_grad():
    pa_t = R.to_t(pa)
    z_ref = R.gnn(pa_t["gnn"], gh, n).reshape(-1, 64 if False else R.gnn(pa_t["gnn"], gh, n).shape[-1])
    y_ref = R.mlp_head(R.gnn(pa_t["gnn"], gh, n), pa_t["head"]).reshape(-1, 64).numpy()
d = np.abs(y_gpu - y_ref).max(1)
print("trunk rows", d.shape[0], "max dev", d.max(), "rows with dev > 1e-5:", np.nonzero(d > 1e-5)[0][:20].tolist())
top = np.argsort(-d)[:8]
for r in top:
    gi, ai = divmod(int(r), n)
    print(f"  row {r} (graph {gi}, agent {ai}) dev {d[r]:.3e}")
# the graph of the worst row: receivers / senders of its valid edges and the node rows
gi = int(np.argmax(d)) // n
N = gh["nodes"].shape[1]
print("worst graph", gi, "N", N, "E", gh["receivers"].shape[1])
print("receivers", gh["receivers"][gi].tolist())
print("senders  ", gh["senders"][gi].tolist())
np.set_printoptions(precision=4, linewidth=220, suppress=True)
print("nodes\n", gh["nodes"][gi])
print("edges\n", gh["edges"][gi])
