"""Multi-update / multi-minibatch checks of the DGPPO update driver (dgppo.py:136-321,
informarl.py:258-457) -- the orchestration the single-minibatch parity tests in test_update_gpu.py
cannot see: which env rows minibatch k gathers, that each minibatch's gradient is taken at the
parameters the previous minibatch's Adam step left, that Adam's moments and step count carry across
minibatches and updates, that the concurrent-stream schedule is bit-identical to the serial one, and
that DGPPO without its safety terms is InforMARL.

* `test_trajectory_matches_oracle_loop`: K = 5 updates x 4 minibatches, teacher-forced: at every
  update the float64 oracle recomputes the prepass (values, GAE targets, merged advantages) from the
  GPU's parameters at the start of that update, and at every minibatch it recomputes the gradient at
  the GPU's parameters before that minibatch, then clip + Adam with the GPU's carried moments; the
  result must equal the parameters the GPU starts the NEXT minibatch (or update) from.  Tolerances as
  in test_update_gpu.py (1e-5 relative + 8x the float32 noise floor of the same oracle; Adam results
  1e-6 absolute).  Teacher forcing keeps the check exact over many steps: an untethered float64 loop
  drifts from any fp32 run within a few Adam steps (sign(g) steps of size lr on near-zero gradients).
* `test_streams_bit_identical`: DGPPO_STREAMS=1 (policy / Vl / Vh passes on three HIP streams) vs 0
  (serial), 3 updates x 8 minibatches: parameters, Adam state and every info entry bit-identical.
* `test_force_safe_dgppo_is_informarl`: DGPPO with cbf_weight 0 and every sample forced safe
  (DGPPO_DEBUG_FORCE_SAFE=1: A = -normalised Al exactly) runs the same policy / Vl update as
  InforMARL with cost_weight 0; 3 updates x 4 minibatches from the same seed, each algorithm
  collecting its own rollouts: policy and Vl parameters agree to 1e-5 (the two advantage kernels
  reduce in different orders, so not bit for bit).
"""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.env import make_env
from oracle import nets as O
from oracle import nets_t as R

from test_update_gpu import _close_floor, _host, _net_trees, _walk

pytestmark = pytest.mark.gpu


def _as64(tree):
    """float64 copy of a gradient tree (dict / list leaves)."""
    if isinstance(tree, dict):
        return {k: _as64(v) for k, v in tree.items()}
    if isinstance(tree, list):
        return [_as64(v) for v in tree]
    return np.asarray(tree, np.float64)


def _algo(cuda, eid, n, obs, T, batch, L=16, algo="dgppo", seed=3, **kw):
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    return make_algo(algo, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=batch, rnn_step=L, train_steps=100, seed=seed,
                     device=cuda, **kw), env


def _trees_at(algo, flats):
    """flax trees of (actor, Vl, Vh) at the given flat parameter vectors (the live buffers are restored)."""
    nets = (("policy", algo.actor), ("Vl", algo.Vl), ("Vh", algo.Vh))
    keep = {k: net.ps.flat.clone() for k, net in nets}
    try:
        for k, net in nets:
            net.ps.flat.copy_(flats[k])
        return _net_trees(algo)
    finally:
        for k, net in nets:
            net.ps.flat.copy_(keep[k])


def _trajectory(cuda, eid, n, obs, K_UPD=5, perturb=None):
    """The teacher-forced K_UPD x 4-minibatch check (module docstring).  `perturb(algo, it, k)` may change the
    algorithm before minibatch k of update it runs (negative controls).  Returns per-minibatch fallback
    records: (update, minibatch, entries over the base tolerance, entries checked, ambiguous gates, gates)."""
    B, T, L = 8, 32, 16
    algo, env = _algo(cuda, eid, n, obs, T, batch=2 * T, L=L)  # 2 envs per minibatch -> 4 minibatches
    nets = (("Vl", algo.Vl), ("Vh", algo.Vh), ("policy", algo.actor))
    if perturb is not None:
        algo._mb_apply = _counting_apply(algo, perturb)
    fallbacks = []
    for it in range(K_UPD):
        algo._traj_it = it
        roll = algo.collect(algo.params, 100 + it, n_env=B)
        start = {k: net.ps.flat.clone() for k, net in nets}
        algo.trace = {}
        step = 20 * it  # crosses the CBF schedule's 50% boundary (train_steps 100) at it = 3
        info = algo.update(roll, step)
        torch.cuda.synchronize()
        tr = algo.trace
        assert len(tr["mb"]) == 4
        hr, hd = _host(roll, n), _host(tr["det"], n)
        cw = algo.cbf_weight_at(step)
        pa, pl, ph = _trees_at(algo, start)
        # prepass at the update-start parameters
        refs = {}
        try:
            for dt in (torch.float64, torch.float32):
                R.T64 = dt
                refs[dt] = R.dgppo_prepass(R.to_t(pa), R.to_t(pl), R.to_t(ph), hr, hd, n, env.dt, algo.gamma,
                                           algo.gae_lambda, algo.alpha, algo.cbf_eps, cw)
        finally:
            R.T64 = torch.float64
        ref, ref32 = refs[torch.float64], refs[torch.float32]
        for k in ("Vl", "Vh", "Ql", "Qh_det"):
            _close_floor(tr[k].cpu().numpy(), ref[k], ref32[k], f"update {it} {k}")
        robust = np.abs(ref["deriv"]).min(-1) > 1e-3
        env_floor = np.broadcast_to(np.abs(ref32["A"] - ref["A"]).max(axis=(1, 2), keepdims=True), ref["A"].shape)
        _close_floor(tr["A"].cpu().numpy()[robust], ref["A"][robust], ref32["A"][robust], f"update {it} A",
                     floor=env_floor[robust])
        # the minibatches partition the envs
        seen = np.sort(np.concatenate([mb["envs"] for mb in tr["mb"]]))
        assert np.array_equal(seen, np.arange(B))
        Ql, Qh_det, A = (tr[k].double().cpu().numpy() for k in ("Ql", "Qh_det", "A"))
        for k, mb in enumerate(tr["mb"]):
            # parameters before minibatch k = start of the update, or Adam after minibatch k - 1
            if k == 0:
                for name, _ in nets:
                    assert torch.equal(mb["before"][name], start[name]), (it, name)
            pa, pl, ph = _trees_at(algo, mb["before"])
            rg = {}
            try:
                for dt in (torch.float64, torch.float32):
                    R.T64 = dt
                    ts = [R.to_t(x, requires_grad=True) for x in (pa, pl, ph)]
                    R.dgppo_minibatch_grads(*ts, hr, hd, np.asarray(mb["envs"]), Ql, Qh_det, A, n, L,
                                            algo.entropy_eps.cpu().numpy(), algo.clip_eps, algo.coef_ent)
                    rg[dt] = [R.grads(t) for t in ts]
            finally:
                R.T64 = torch.float64
            keep = algo.grad_flat.clone()
            algo.grad_flat.copy_(mb["grad"])
            gpu = _net_trees(algo, grad=True)
            algo.grad_flat.copy_(keep)
            gate_floor = None  # effect of the ReLU gates fp32 rounding decides, computed on demand
            gate_stats = []
            r64_leaves = rg[torch.float64]

            def gate_floors():
                # |on - off| + |on - natural| + |off - natural| per entry: one ambiguous gate's effect is |on - off|;
                # the one-sided toggles bound mixed decisions over several ambiguous gates
                out = [r64_leaves]
                R.GATE_STATS = gate_stats
                try:
                    for mode in ("on", "off"):
                        R.GATE_MODE = mode
                        ts = [R.to_t(x, requires_grad=True) for x in (pa, pl, ph)]
                        R.dgppo_minibatch_grads(*ts, hr, hd, np.asarray(mb["envs"]), Ql, Qh_det, A, n, L,
                                                algo.entropy_eps.cpu().numpy(), algo.clip_eps, algo.coef_ent)
                        out.append([R.grads(t) for t in ts])
                finally:
                    R.GATE_MODE = None
                    R.GATE_STATS = None
                nat, on, off = out
                return [[np.abs(x - y) + np.abs(x - z) + np.abs(y - z) for (_, x, y), (_, _, z) in
                         zip(_walk(_as64(a), _as64(b)), _walk(_as64(a), _as64(c)))] for a, b, c in zip(on, off, nat)]

            n_over = n_checked = 0
            for ti, (tag, g, r64, r32) in enumerate(zip(("actor", "Vl", "Vh"), gpu, rg[torch.float64], rg[torch.float32])):
                for li, ((path, a, b), (_, c, _)) in enumerate(zip(_walk(g, r64), _walk(r32, r64))):
                    b = np.asarray(b, np.float64)
                    d = np.abs(np.asarray(a, np.float64) - b)
                    floor = np.abs(np.asarray(c, np.float64) - b).max()
                    tol = 2e-5 * np.abs(b).max() + 1e-6 + 8 * floor
                    n_checked += d.size
                    if d.max() > tol:
                        # entries whose float64 value hangs on a ReLU gate within fp32 rounding of zero: either
                        # decision is a correct fp32 result, so those entries may differ by the gate's effect
                        n_over += int((d > tol).sum())
                        gate_floor = gate_floor or gate_floors()
                        tol = tol + gate_floor[ti][li]
                    err = d.max()
                    worst = np.unravel_index(np.argmax(d - tol), d.shape)
                    assert (d <= tol).all(), \
                        (f"update {it} mb {k} {tag} grad {path}: {err:.3e} (fp32 floor {floor:.3e}); "
                         f"{int((d > tol).sum())} of {d.size} entries over, worst at {np.unravel_index(d.argmax(), d.shape)} "
                         f"gpu {np.asarray(a).ravel()[d.argmax()]:.6e} ref {b.ravel()[d.argmax()]:.6e}, "
                         f"median err {np.median(d):.2e}, fp32 oracle {np.asarray(c, np.float64).ravel()[d.argmax()]:.6e}, "
                         f"gate floor {0.0 if gate_floor is None else gate_floor[ti][li].ravel()[d.argmax()]:.3e}; "
                         f"largest excess at {worst}: err {d[worst]:.3e} tol {np.broadcast_to(tol, d.shape)[worst]:.3e}")
            amb, gates = sum(x for x, _ in gate_stats), sum(y for _, y in gate_stats)
            fallbacks.append((it, k, n_over, n_checked, amb, gates))
            # clip + Adam with the carried moments -> the parameters the next minibatch starts from: every entry within
            # 1e-6, and the Adam STEP itself to 1e-4 relative (median over the entries whose step is resolvable in fp32:
            # |p| < 0.05 and |step| > 0.1 lr; an fp32 step is ~1e-6 relative off, a moment update that cancels can be
            # far more, hence the median) -- tight enough that a 0.1% learning-rate error in one minibatch fails
            # (test_trajectory_negative_control)
            nxt = tr["mb"][k + 1]["before"] if k + 1 < len(tr["mb"]) else {nm: net.ps.flat for nm, net in nets}
            off = 0
            for name, net in nets:
                sz = net.ps.size
                g = mb["grad"][off:off + sz].double().cpu().numpy()
                off += sz
                (gc,), _ = O.clip_by_global_norm_ref([g], algo.max_grad_norm)
                count = int(mb["state_before"][name][2].item())
                assert count == it * 4 + k, (it, k, name, count)  # every step so far was finite
                lr = algo.opt[name].__dict__.get("lr_ref", algo.opt[name].lr)
                (rp,), _, _ = O.adam_step([mb["before"][name].double().cpu().numpy()], [gc],
                                          [mb["m_before"][name].double().cpu().numpy()],
                                          [mb["v_before"][name].double().cpu().numpy()], count, lr)
                got = nxt[name].double().cpu().numpy()
                p0 = mb["before"][name].double().cpu().numpy()
                err = np.abs(got - rp)
                assert err.max() <= 1e-6, f"update {it} mb {k} {name} Adam: {err.max():.3e}"
                step_ref, step_gpu = rp - p0, got - p0
                sel = (np.abs(p0) < 0.05) & (np.abs(step_ref) > 0.1 * lr)
                if sel.sum() >= 20:
                    rel = np.median(np.abs(step_gpu[sel] - step_ref[sel]) / np.abs(step_ref[sel]))
                    assert rel <= 1e-4, f"update {it} mb {k} {name} Adam step: median relative error {rel:.2e} over {sel.sum()}"
        assert np.isfinite(info["policy/loss"])
    return fallbacks


def _counting_apply(algo, perturb):
    """algo._mb_apply wrapped so perturb(algo, opt, name, update, minibatch) runs for every net before each minibatch's
    clip + Adam launch (the per-net pairs or the multi-net kernel read each optimiser's lr at that point)."""
    orig = algo._mb_apply
    algo._mb_count = -1

    def apply():
        algo._mb_count += 1
        for name, opt in algo.opt.items():
            perturb(algo, opt, name, getattr(algo, "_traj_it", 0), algo._mb_count % 4)
        orig()
    return apply


@pytest.mark.parametrize("eid,n,obs", [("LidarSpread", 3, 2), ("MPETarget", 2, 0)])
def test_trajectory_matches_oracle_loop(cuda, eid, n, obs):
    fb = _trajectory(cuda, eid, n, obs)
    # the gate fallback is bounded: at most 0.1% of the ReLU gates a minibatch evaluates may be decided by fp32
    # rounding, and at most a quarter of the minibatches may need the fallback at all (the rounds so far: 0 or 1
    # of 20); every count is printed (pytest -s / the log on failure)
    for it, k, n_over, n_checked, amb, gates in fb:
        print(f"{eid} update {it} mb {k}: {n_over} of {n_checked} gradient entries over the base tolerance; "
              f"{amb} ambiguous of {gates} ReLU gates")
        assert amb <= max(2, 1e-3 * gates), (it, k, amb, gates)
    used = sum(1 for r in fb if r[2] > 0)
    assert used <= len(fb) // 4, f"{used} of {len(fb)} minibatches needed the gate fallback"


def test_trajectory_negative_control(cuda):
    """A 0.1% learning-rate error in ONE minibatch's policy Adam step (update 0, minibatch 1) must fail the
    trajectory check: the teacher-forced comparison is sensitive to a real orchestration error of that size."""
    def perturb(algo, opt, name, it, k):
        if name == "policy":
            opt.lr_ref = opt.__dict__.get("lr_ref", opt.lr)
            opt.lr = opt.lr_ref * (1.001 if (it, k) == (0, 1) else 1.0)

    with pytest.raises(AssertionError, match="mb 1 policy Adam"):
        _trajectory(cuda, "LidarSpread", 3, 2, K_UPD=1, perturb=perturb)


def test_streams_bit_identical(cuda, monkeypatch):
    eid, n, obs, B, T = "LidarSpread", 3, 2, 8, 32

    def run(flag):
        monkeypatch.setenv("DGPPO_STREAMS", flag)
        algo, _ = _algo(cuda, eid, n, obs, T, batch=T)  # 1 env per minibatch -> 8 minibatches
        infos = []
        for it in range(3):
            infos.append(algo.update(algo.collect(algo.params, 21 + it, n_env=B), it))
        torch.cuda.synchronize()
        return algo, infos

    a1, i1 = run("1")
    assert a1._aux_streams(2) is not None
    a0, i0 = run("0")
    assert a0._aux_streams(2) is None
    for name in ("Vl", "Vh", "policy"):
        o0, o1 = a0.opt[name], a1.opt[name]
        assert torch.equal(o0.ps.flat, o1.ps.flat), name
        assert torch.equal(o0.m, o1.m) and torch.equal(o0.v, o1.v) and torch.equal(o0.state, o1.state), name
    for d0, d1 in zip(i0, i1):
        assert d0.keys() == d1.keys()
        for k in d0:
            assert d0[k] == d1[k] or (np.isnan(d0[k]) and np.isnan(d1[k])), k


def test_force_safe_dgppo_is_informarl(cuda, monkeypatch):
    eid, n, obs, B, T = "LidarTarget", 2, 1, 8, 32
    monkeypatch.setenv("DGPPO_DEBUG_FORCE_SAFE", "1")
    dg, _ = _algo(cuda, eid, n, obs, T, batch=2 * T, cbf_weight=0.0)
    inf, _ = _algo(cuda, eid, n, obs, T, batch=2 * T, algo="informarl", cost_weight=0.0)
    for name in ("policy", "Vl"):
        assert torch.equal(dg.params[name], inf.params[name])
    for it in range(3):
        rd = dg.collect(dg.params, 40 + it, n_env=B)
        ri = inf.collect(inf.params, 40 + it, n_env=B)
        assert (rd.actions - ri.actions).abs().max().item() <= 1e-5, it
        idg = dg.update(rd, it)
        iinf = inf.update(ri, it)
        assert idg["eval/safe_data"] == 1.0
        for name in ("policy", "Vl"):
            err = (dg.params[name] - inf.params[name]).abs().max().item()
            assert err <= 1e-5, f"update {it} {name}: {err:.3e}"
        for k in ("Vl/loss", "policy/loss", "policy/entropy", "policy/clip_frac"):
            assert abs(idg[k] - iinf[k]) <= 1e-5 * (1 + abs(iinf[k])), (it, k, idg[k], iinf[k])
