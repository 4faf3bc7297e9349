"""Analytic flop count of one DGPPO update in the formulation the kernels implement (per-receiving-
agent attention with Q-free projections, never-receivers' layer-1 rows recomputed from the raw rows), replacing
SURVEY.md §8(d)'s node-level-projection count.  Reference composition: `dgppo.py:203-228`
(prepass: Vl scan, Vh on the rollout and on the deterministic rollout, whose actor inference is counted too) and
`dgppo.py:275-289` (every graph once through the three nets' forward + backward per PPO epoch).

Counting rules (2 flops per multiply-add; the same rules for every net):
* a dense product y = x W (m rows, k in, f out): forward 2 m k f; backward 2 m k f for dW, plus 2 m k f for dx
  unless x is a raw graph row (no gradient flows into the environment's features);
* per receiving agent r, head h and candidate c of a GraphTransformer layer (`gnn.py:86-111`): the logit
  qt_h . x_c (2 D), the softmax (5 per element: max, subtract, exp, sum, divide; backward 4), the weighted sums
  of the candidate rows and edge features (2 (D + 5): D row columns, 4 edge columns, the weight itself);
  backward of both bilinear terms = 2 x forward, 1 x where the candidate rows are raw rows;
* [qt | beta] = [x 1] QBW per receiver (2 (D + 1) H (D + 1)), the message GEMM xcat Wcat / H (2 H (D + 5) F),
  the update x Wu + bu (2 D F); layer l >= 2 of the reference's 2-layer GNNs recomputes each never-receiving
  node's layer-1 row once (2 D0 D per node, backward: dW only);
* MLP head 2 x Dense(64, 64) (LayerNorm / ReLU elementwise, not counted), GRU 2 x 64 x 3 x 64 per row for the
  input projection and again for the recurrence (LSTM: 4 gates), the output Dense layers.
Elementwise work (LayerNorm, ReLU, GRU gates, tanh-normal, Adam, GAE) is not counted: it is < 1% of the total."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class GraphShape:
    n: int  # receiving agents per graph
    C: int  # candidate senders per receiver (agents + goal edges + lidar hits / obstacles)
    N_nr: int  # never-receiving sender nodes per graph (goals, hits, obstacles; the pad node excluded)
    D0: int  # raw node row width


def graph_shape(env) -> GraphShape:
    cand = env.agent_candidates("cpu")
    n, C = int(cand.shape[0]), int(cand.shape[1])
    N = int(env.num_nodes) if hasattr(env, "num_nodes") else None
    if N is None:
        g = env.empty_graph(1, device="cpu")
        N = int(g.nodes.shape[-2])
    return GraphShape(n, C, N - n - 1, int(env.node_dim))


def _dense(m, k, f, dx=True):
    fwd = 2.0 * m * k * f
    return fwd, fwd * (2.0 if dx else 1.0)


def gnn_layer(gs: GraphShape, D, F, H, EX, first: bool, agent_mode: bool, D0_pre: int | None):
    """(forward, backward) flops of one GraphTransformer layer per graph."""
    n, C = gs.n, gs.C
    f = b = 0.0
    raw_in = first  # layer 0 reads the raw rows: no gradient into them
    for fw, bw in (_dense(n, D + 1, H * D + H, dx=not raw_in),  # [qt | beta]
                   _dense(n, H * (D + 5 + EX), F),  # message GEMM (+ the Wex columns)
                   _dense(n, D, F, dx=not raw_in)):  # update
        f, b = f + fw, b + bw
    pairs = n * H * C
    bil = 2.0 * pairs * D + 2.0 * pairs * (D + 5 + EX)
    f += bil + 5.0 * pairs
    b += bil * (1.0 if raw_in else 2.0) + 4.0 * pairs
    if agent_mode and D0_pre:  # never-receivers' layer-1 rows from the raw rows, once per node
        fw = 2.0 * gs.N_nr * D0_pre * D
        f, b = f + fw, b + fw
    return f, b


def net_per_graph(net, gs: GraphShape, kind: str):
    """(forward, backward) flops per graph of ActorNet / VlNet / VhNet as the kernels run them.  kind: "actor",
    "Vl" (agent mean before the head: head / RNN / out on one row per graph), "Vh"."""
    f = b = 0.0
    layers = net.gnn.layers
    for i, L in enumerate(layers):
        fw, bw = gnn_layer(gs, L.D, L.F, L.H, L.EX, first=(i == 0), agent_mode=(i == 1),
                           D0_pre=layers[0].D if i == 1 else None)
        f, b = f + fw, b + bw
    rows = 1 if kind == "Vl" else gs.n
    dense = [(64, 64), (64, 64)]  # MLP head
    for c in net.gru.cells:
        gates = 4 if type(c).__name__ == "LSTMCell" else 3
        dense += [(c.d_in, gates * c.H), (c.H, gates * c.H)]
    if kind == "actor":
        dense += [(64, 64), (64, 2 * net.mean.d_out)]  # ScaleHid, mean + std
    else:
        dense += [(64, net.out.d_out)]
    for k, fo in dense:
        fw, bw = _dense(rows, k, fo)
        f, b = f + fw, b + bw
    return f, b


def update_flops(algo, env, n_env: int, T: int) -> dict:
    """Flops of one DGPPO.update over n_env envs x T steps (epoch_ppo passes of SGD), by part, and the total."""
    gs = graph_shape(env)
    G = float(n_env * T)
    a = net_per_graph(algo.actor, gs, "actor")
    vl = net_per_graph(algo.Vl, gs, "Vl")
    vh = net_per_graph(algo.Vh, gs, "Vh")
    ep = float(getattr(algo, "epoch_ppo", 1))
    parts = {
        "det_rollout_actor": G * a[0],
        "prepass_Vl": G * vl[0],
        "prepass_Vh_rollout_and_det": 2.0 * G * vh[0],
        "sgd_fwd_bwd": ep * G * (a[0] + a[1] + vl[0] + vl[1] + vh[0] + vh[1]),
    }
    per_graph = {"actor": a, "Vl": vl, "Vh": vh}
    return {"total": sum(parts.values()), "parts": parts,
            "per_graph_fwd_mflop": {k: round(v[0] / 1e6, 4) for k, v in per_graph.items()},
            "per_graph_bwd_mflop": {k: round(v[1] / 1e6, 4) for k, v in per_graph.items()}}
