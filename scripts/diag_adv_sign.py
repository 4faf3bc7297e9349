"""Diagnostic: is the advantage positive for goal-directed actions?

Collects a LidarTarget (own goal per agent) rollout with the untrained policy and correlates the
traced InforMARL/DGPPO advantage A[b, t, i] with the goal-directed component of the action,
a . (goal - pos) / |goal - pos| (double integrator: the action is an acceleration).  Moving toward the
goal lowers the future cost-to-go, so a correctly signed advantage correlates positively."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    algo_name = sys.argv[1] if len(sys.argv) > 1 else "informarl"
    env_id = sys.argv[2] if len(sys.argv) > 2 else "LidarTarget"
    n = 4
    env = make_env(env_id, n, num_obs=0 if env_id.startswith("MPE") else 2, device=dev)
    B, T, L = 128, env.max_episode_steps, 16
    algo = make_algo(algo_name, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T, rnn_step=L, seed=0, device=dev)
    roll = algo.collect(algo.params, 5, n_env=B)
    st = roll.graph.states.cpu().numpy()  # (B, T, N, sd)
    pos, vel, goal = st[:, :, :n, :2], st[:, :, :n, 2:4], st[:, :, n:2 * n, :2]
    acts = roll.actions.cpu().numpy()  # (B, T, n, 2)
    algo.trace = {}
    algo.update(roll, 0)
    A = algo.trace["A"].cpu().numpy()  # (B, T, n)
    Ql, Vl = algo.trace["Ql"].cpu().numpy(), algo.trace["Vl"].cpu().numpy()
    d = goal - pos
    u = d / (np.linalg.norm(d, axis=-1, keepdims=True) + 1e-9)
    toward = (acts * u).sum(-1)  # goal-directed acceleration
    vtoward = (vel * u).sum(-1)
    c = lambda x, y: float(np.corrcoef(x.reshape(-1), y.reshape(-1))[0, 1])  # noqa: E731
    rew = roll.rewards.cpu().numpy()
    print(f"{algo_name} {env_id}: corr(A, a.toward_goal) = {c(A, toward):+.4f}   corr(A, v.toward_goal) = "
          f"{c(A, vtoward):+.4f}")
    # time alignment of the targets: Ql[t] - gamma Ql[t+1] should be l[t] = -reward[t] (lambda = 1 part)
    dist = np.linalg.norm(d, axis=-1).mean(-1)  # (B, T)
    print(f"corr(-reward[t], mean dist[t]) = {c(-rew, dist):+.4f}  corr(Ql[t], mean dist[t]) = {c(Ql, dist):+.4f}  "
          f"corr(Vl[t], mean dist[t]) = {c(Vl[:, :T], dist):+.4f}")
    # one-step effect: moving toward the goal at t reduces the distance at t+1
    ddist = dist[:, 1:] - dist[:, :-1]
    print(f"corr(mean toward[t], dist[t+1]-dist[t]) = {c(toward[:, :-1].mean(-1), ddist):+.4f}")


if __name__ == "__main__" and (len(sys.argv) < 2 or sys.argv[1] not in ("trend", "consistency")):
    main()


def trend():
    """Advantage structure over time and its correlation with simple action features."""
    dev = torch.device("cuda", 0)
    env_id = sys.argv[2] if len(sys.argv) > 2 else "LidarTarget"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    env = make_env(env_id, n, num_obs=0, device=dev)
    B, T, L = 128, env.max_episode_steps, 16
    algo = make_algo("informarl", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T, rnn_step=L, seed=0, device=dev)
    for it in range(40):
        roll = algo.collect(algo.params, 5 + it, n_env=B)
        algo.trace = {}
        info = algo.update(roll, it)
        if it % 4:
            continue
        A = algo.trace["A"].cpu().numpy()[..., 0]  # (B, T)
        Ql, Vl = algo.trace["Ql"].cpu().numpy(), algo.trace["Vl"].cpu().numpy()
        acts = roll.actions.cpu().numpy()
        st = roll.graph.states.cpu().numpy()
        speed = np.linalg.norm(st[:, :, :n, 2:4], axis=-1).mean(-1)
        rew = roll.rewards.cpu().numpy()
        c = lambda x, y: float(np.corrcoef(x.reshape(-1), y.reshape(-1))[0, 1])  # noqa: E731
        tt = np.broadcast_to(np.arange(T)[None], (B, T))
        print(f"it {it:2d}: ep reward {rew.sum(1).mean():+.3f}  mean a {acts.mean((0, 1, 2))}  corr(A,t) {c(A, tt):+.3f}"
              f"  corr(Ql-Vl,t) {c(Ql - Vl[:, :T], tt):+.3f}  corr(A, speed) {c(A, speed):+.3f}  "
              f"corr(A, mean a_x) {c(A, acts[..., 0].mean(-1)):+.3f}  corr(A, mean a_y) {c(A, acts[..., 1].mean(-1)):+.3f}"
              f"  Vl[0] {Vl[:, 0].mean():.3f} Ql[0] {Ql[:, 0].mean():.3f} Vl[T] {Vl[:, T].mean():.3f} "
              f"Ql[T-1] {Ql[:, T - 1].mean():.3f}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "trend":
    trend()


def consistency():
    """Rollout policy (fused kernel, carried GRU state) vs the update's policy evaluation (unfused,
    one 128-step chunk from a zero carry = exactly the rollout's carries): log pi of the stored actions."""
    dev = torch.device("cuda", 0)
    env = make_env("LidarSpread", 8, num_obs=3, device=dev)
    B, T = 64, env.max_episode_steps
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=8, batch_size=B * T, rnn_step=16, seed=0, device=dev)
    for it in range(31):
        roll = algo.collect(algo.params, 7 + it, n_env=B)
        if it % 10 == 0:
            g = algo._graphs(roll.graph, slice(None))
            acts = roll.actions.reshape(-1, 2).contiguous()
            lp, _, _ = algo.actor.eval_seq_fwd(g, B, T, acts, algo.entropy_eps)
            old = roll.log_pis.reshape(-1)
            d = (lp - old).abs()
            lp16, _, _ = algo.actor.eval_seq_fwd(g, B * T // 16, 16, acts, algo.entropy_eps)
            d16 = (lp16 - old).abs()
            print(f"it {it}: |log pi(eval, 1 chunk) - log pi(rollout)| max {d.max():.3e} mean {d.mean():.3e}; "
                  f"16-step chunks: max {d16.max():.3e} mean {d16.mean():.3e}; sat frac "
                  f"{(acts.abs() > 0.999).float().mean():.3f}", flush=True)
        algo.update(roll, it)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "consistency":
    consistency()
