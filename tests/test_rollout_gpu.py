"""GPU parity for the policy rollout (trainer/utils.py:22-86 rollout / test_rollout as one
captured hipGraph, trainer/rollout.py): every step's actor carry, tanh-normal action and log_pi
against the float64 oracle (policy.py:61-74, 191-212, distribution.py), the env transition
against the env kernel itself (bit-exact), and the carry-storage conventions of both rollouts.

The sampling noise is the framework's Philox stream (the reference's threefry stream is not
reproducible without JAX), regenerated here from (key, env_offset, t); its moments are checked.
Tolerances: carries / actions / log_pi |gpu - ref| <= 3e-5 (1 + |ref|)."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.env import make_env
from dgppo_fov_amd.nn import kernels as K
from dgppo_fov_amd.trainer.rollout import RolloutEngine
from oracle import nets_t as R

pytestmark = pytest.mark.gpu


def _close(a, b, tol, what):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = (np.abs(a - b) - tol * (1 + np.abs(b))).max()
    assert err <= 0, f"{what}: max abs err {np.abs(a - b).max():.3e}"


def test_normal_moments(cuda):
    x = torch.empty(1 << 22, device=cuda)
    K.normal_(x, seed=123, stream_id=5)
    y = x.double()
    assert abs(y.mean().item()) < 3e-3 and abs(y.std().item() - 1) < 3e-3
    assert abs((y ** 4).mean().item() - 3) < 2e-2
    z = torch.empty_like(x)
    K.normal_(z, seed=123, stream_id=6)
    assert abs(torch.corrcoef(torch.stack([x, z]))[0, 1].item()) < 3e-3
    z2 = torch.empty_like(x)
    K.normal_(z2, seed=123, stream_id=5)
    assert torch.equal(x, z2)


def _host_graph(eng, t):
    b = eng.buf
    return {k: getattr(b, k)[t].cpu().numpy() for k in ("nodes", "edges", "receivers", "senders")}


@pytest.mark.parametrize("eid,n,obs,graph", [("LidarSpread", 3, 2, True), ("MPETarget", 3, 0, False),
                                             ("LidarBicycleTarget", 2, 1, True), ("LidarOmniTarget", 3, 2, True)])
def test_policy_rollout_matches_oracle(cuda, eid, n, obs, graph):
    B, T = 3, 12
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T, rnn_step=4, seed=2, device=cuda)
    pa = R.to_t(algo.actor.flax())
    for mode in (RolloutEngine.MODE_SAMPLE, RolloutEngine.MODE_DET):
        eng = RolloutEngine(env, B, T, cuda, env_offset=0, actor=algo.actor, mode=mode)
        if graph:
            eng.capture()
        roll = eng.run(11)
        torch.cuda.synchronize()
        rnn = eng.rnn.cpu().numpy()
        assert np.abs(rnn[0]).max() == 0
        noise = torch.empty((B * n, env.action_dim), device=cuda)
        for t in range(T):
            g = _host_graph(eng, t)
            with torch.no_grad():
                h2 = R.actor_carry(pa, g, rnn[t], n)
                mu, sd = R.policy_dist(pa, h2)
            _close(rnn[t + 1], h2.numpy(), 3e-5, f"carry t={t}")
            a = eng.actions[t].cpu().numpy()
            if mode == RolloutEngine.MODE_SAMPLE:
                K.normal_(noise, seed=11, stream_id=t)
                eps = noise.view(B, n, -1).double().cpu()
                _close(a, torch.tanh(mu + sd * eps).numpy(), 3e-5, f"action t={t}")
                lp = R.tanh_normal_log_prob(a.astype(np.float64), mu, sd)
                _close(eng.log_pis[t].cpu().numpy(), lp.numpy(), 3e-5, f"log_pi t={t}")
            else:
                _close(a, torch.tanh(mu).numpy(), 3e-5, f"det action t={t}")
            # env transition: graph t+1 is exactly env.step(graph t, action t)
            nxt = env.step(eng.graph_at(t), eng.actions[t])
            for k in ("nodes", "edges", "states", "receivers", "senders"):
                assert torch.equal(getattr(nxt.graph, k), getattr(eng.graph_at(t + 1), k)), (t, k)
            assert torch.equal(nxt.reward, eng.rewards[t]) and torch.equal(nxt.cost, eng.costs[t])
        # storage conventions (utils.py:186-192 stochastic: carry before; 211-218 det: carry after)
        want = slice(0, T) if mode == RolloutEngine.MODE_SAMPLE else slice(1, T + 1)
        got = roll.rnn_states.reshape(B, T, n, 64).transpose(0, 1).cpu().numpy()
        assert np.array_equal(got, rnn[want])
        assert roll.graph.nodes.shape[:2] == (B, T) and roll.next_graph.nodes.shape[:2] == (B, T)
        assert torch.equal(roll.next_graph.nodes[:, 0], roll.graph.nodes[:, 1])


def test_rollout_shards_use_disjoint_noise(cuda):
    env = make_env("MPETarget", 3, num_obs=0, max_step=4, device=cuda)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=3, batch_size=8, rnn_step=4, seed=2, device=cuda)
    acts = []
    for off in (0, 2):
        eng = RolloutEngine(env, 2, 4, cuda, env_offset=off, actor=algo.actor, mode=RolloutEngine.MODE_SAMPLE)
        eng.run(5)
        acts.append(eng.actions.clone())
    assert not torch.equal(acts[0], acts[1])


@pytest.mark.parametrize("eid,n,obs", [("LidarSpread", 8, 3), ("LidarOmniTarget", 3, 2)])
def test_policy_step_in_kernel_noise_bit_exact(cuda, eid, n, obs):
    """ABI 10: the fused policy step drawing its Philox noise in the kernel (noise_seed, noise_stream) gives the
    same action, log_pi and carry bits as the step fed the buffer dgppo_normal writes for that stream."""
    B = 37
    env = make_env(eid, n, num_obs=obs, max_step=4, device=cuda)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=8, rnn_step=4, seed=3, device=cuda)
    eng = RolloutEngine(env, B, 4, cuda, env_offset=0, actor=algo.actor, mode=RolloutEngine.MODE_DET)
    eng.run(9)
    g = eng._batch(2)
    h = torch.randn((B * n, 64), generator=torch.Generator().manual_seed(4)).to(cuda)
    key = torch.tensor([0x1234_5678_9ABC], dtype=torch.int64, device=cuda)
    sid = (5 << 32) | 7
    noise = torch.empty((B * n, env.action_dim), device=cuda)
    K.normal_(noise, stream_id=sid, seed_tensor=key)
    ref = algo.actor.act(g, h, 1, noise=noise)
    got = algo.actor.act(g, h, 1, noise=torch.full_like(noise, float("nan")), noise_seed=key, noise_stream=sid)
    torch.cuda.synchronize()
    for a, b, what in zip(ref, got, ("action", "log_pi", "carry")):
        assert torch.equal(a, b), what


@pytest.mark.parametrize("graph", [False, True])
def test_env_rollout_lanes_bit_exact(cuda, graph):
    """Env-only rollout stepped as 2 env slices on 2 streams (RolloutEngine lanes=2) writes the same
    (T+1, B) buffer, rewards and costs as the single-stream rollout, bit for bit."""
    env = make_env("LidarSpread", 8, num_obs=3, device=cuda)
    B, T = 256, 12
    outs = []
    for lanes in (1, 2):
        eng = RolloutEngine(env, B, T, cuda, lanes=lanes)
        gen = torch.Generator(device=cuda)
        gen.manual_seed(5)
        eng.actions.uniform_(-1.0, 1.0, generator=gen)
        if graph:
            eng.capture()
        eng.run(key=3)
        torch.cuda.synchronize(cuda)
        b = eng.buf
        outs.append([x.cpu().numpy() for x in (b.nodes, b.edges, b.states, b.receivers, b.senders,
                                              eng.rewards, eng.costs)])
    for x, y in zip(*outs):
        assert np.array_equal(x, y)
    with pytest.raises(ValueError):
        RolloutEngine(env, 255, T, cuda, lanes=2)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("env_id", ["LidarSpread", "LidarOmniTarget"])
def test_policy_rollout_lanes_bit_exact(cuda, env_id, graph):
    """Policy rollouts (sample and det) stepped as 2 env slices on 2 streams write the same actions,
    log_pi, carries and graphs as one stream, bit for bit, replayed from a hipGraph and eager
    (LidarOmniTarget through the wide instantiation of the fused policy step: 10-wide nodes / edges, 3 actions)."""
    env = make_env(env_id, 8, num_obs=3, device=cuda)
    B, T = 64, 6
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=8, batch_size=B * T, rnn_step=3, seed=4, device=cuda)
    for mode in (RolloutEngine.MODE_SAMPLE, RolloutEngine.MODE_DET):
        outs = []
        for lanes in (1, 2):
            eng = RolloutEngine(env, B, T, cuda, env_offset=0, actor=algo.actor, mode=mode, lanes=lanes)
            if lanes == 2:
                assert eng.lanes == 2
            if graph:
                eng.capture()
            eng.run(key=11)
            torch.cuda.synchronize(cuda)
            outs.append([x.cpu().numpy() for x in (eng.buf.states, eng.buf.edges, eng.actions, eng.log_pis,
                                                  eng.rnn, eng.rewards, eng.costs)])
        for x, y in zip(*outs):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("eid,n,obs,B", [("LidarSpread", 8, 3, 255), ("LidarTarget", 8, 3, 64),
                                         ("LidarBicycleTarget", 8, 3, 130), ("LidarOmniTarget", 8, 3, 97),
                                         ("MPESpread", 3, 3, 33), ("MPETarget", 3, 3, 29), ("LidarSpread", 4, 2, 20),
                                         # the workgroup-per-env persistent kernel (env_rollout_block_kernel)
                                         ("MPETarget", 3, 0, 17), ("LidarTarget", 2, 0, 11),
                                         ("LidarBicycleTarget", 2, 1, 7), ("LidarSpread", 32, 8, 5)])
@pytest.mark.parametrize("graph", [False, True])
def test_persistent_env_rollout_bit_exact(cuda, eid, n, obs, B, graph):
    """The env-only rollout as ONE persistent launch (states-only reset + dgppo_env_rollout, a wave per
    env for all T steps with its state in LDS) writes the same (T+1, B) graphs, rewards and costs as
    reset + T single-step launches, bit for bit -- also for partial workgroups and, through the
    per-step fallback, configs without the persistent kernel."""
    env = make_env(eid, n, num_obs=obs, device=cuda)
    T = 24
    outs = []
    for fused in (False, True):
        eng = RolloutEngine(env, B, T, cuda, fused=fused)
        gen = torch.Generator(device=cuda)
        gen.manual_seed(9)
        eng.actions.uniform_(-1.2, 1.2, generator=gen)  # includes out-of-range actions (clipped)
        if graph:
            eng.capture()
        eng.run(key=21)
        torch.cuda.synchronize(cuda)
        b = eng.buf
        outs.append([x.cpu().numpy() for x in (b.nodes, b.edges, b.states, b.receivers, b.senders, eng.rewards,
                                              eng.costs)])
    for k, (x, y) in enumerate(zip(*outs)):
        assert np.array_equal(x, y), k


@pytest.mark.parametrize("eid,n,obs,B,T", [
    ("MPESpread", 3, 3, 9, 128),     # T * 2n = 768 action floats: staged in LDS at kernel start
    ("MPESpread", 3, 3, 9, 700),     # 4200 > kActStage: per-step action prefetch from HBM
    ("LidarSpread", 32, 8, 3, 128),  # 8192 > kActStage (the default n = 32 episode): prefetch path
    ("LidarSpread", 32, 8, 3, 24),   # 1536 fits kActStage and 37.3 KB of carve + 6 KB <= 64 KB: staged
])
def test_persistent_block_rollout_action_staging_branches(cuda, eid, n, obs, B, T):
    """Both branches of the block persistent rollout's action staging (the host decides it from kActStage and
    the 64 KB dynamic-LDS budget) match T single-step launches bit for bit, at the default T = 128 too."""
    env = make_env(eid, n, num_obs=obs, device=cuda)
    outs = []
    for fused in (False, True):
        eng = RolloutEngine(env, B, T, cuda, fused=fused)
        gen = torch.Generator(device=cuda)
        gen.manual_seed(5)
        eng.actions.uniform_(-1.2, 1.2, generator=gen)
        eng.run(key=17)
        torch.cuda.synchronize(cuda)
        b = eng.buf
        outs.append([x.cpu().numpy() for x in (b.nodes, b.edges, b.states, b.receivers, b.senders, eng.rewards,
                                              eng.costs)])
    for k, (x, y) in enumerate(zip(*outs)):
        assert np.array_equal(x, y), k


def test_block_persistent_rollout_matches_wave_steps(cuda):
    """With the workgroup-per-env kernels forced (dgppo_env_set_step_kernel(1)), the n = 8 Lidar configs take the
    block persistent rollout; it matches the default path (wave kernels) bit for bit."""
    from dgppo_fov_amd import _lib
    lib = _lib.load()
    env = make_env("LidarSpread", 8, num_obs=3, device=cuda)
    B, T = 37, 16
    outs = []
    for mode in (0, 1):
        prev = lib.dgppo_env_set_step_kernel(mode)
        try:
            eng = RolloutEngine(env, B, T, cuda, fused=True)
            gen = torch.Generator(device=cuda)
            gen.manual_seed(3)
            eng.actions.uniform_(-1.0, 1.0, generator=gen)
            eng.run(key=8)
            torch.cuda.synchronize(cuda)
            b = eng.buf
            outs.append([x.cpu().numpy() for x in (b.nodes, b.edges, b.states, b.receivers, b.senders, eng.rewards,
                                                  eng.costs)])
        finally:
            lib.dgppo_env_set_step_kernel(prev)
    for k, (x, y) in enumerate(zip(*outs)):
        assert np.array_equal(x, y), k


@pytest.mark.parametrize("eid", ["MPESpread", "MPETarget"])
def test_mpe_wave_rollout_matches_block_rollout(cuda, eid):
    """MPE n = 3 with 3 obstacles (BASELINE config 2) runs the wave-per-env persistent rollout
    (wv::mpew::mpe_rollout_wave_kernel); with the workgroup-per-env kernels forced it runs the block persistent
    rollout: the two agree bit for bit at the episode length, partial workgroups and out-of-range actions included."""
    from dgppo_fov_amd import _lib
    lib = _lib.load()
    env = make_env(eid, 3, num_obs=3, device=cuda)
    B, T = 45, 128
    outs = []
    for mode in (0, 1):
        prev = lib.dgppo_env_set_step_kernel(mode)
        try:
            eng = RolloutEngine(env, B, T, cuda, fused=True)
            gen = torch.Generator(device=cuda)
            gen.manual_seed(13)
            eng.actions.uniform_(-1.3, 1.3, generator=gen)
            eng.run(key=31)
            torch.cuda.synchronize(cuda)
            b = eng.buf
            outs.append([x.cpu().numpy() for x in (b.nodes, b.edges, b.states, b.receivers, b.senders, eng.rewards,
                                                  eng.costs)])
        finally:
            lib.dgppo_env_set_step_kernel(prev)
    for k, (x, y) in enumerate(zip(*outs)):
        assert np.array_equal(x, y), k


def test_persistent_env_rollout_from_a_loaded_graph(cuda):
    """rebuild_first = False: the kernel loads graph 0's rows (a full reset) instead of rebuilding them."""
    env = make_env("LidarSpread", 8, num_obs=3, device=cuda)
    B, T = 64, 10
    ref = RolloutEngine(env, B, T, cuda, fused=False)
    ref.actions.uniform_(-1, 1)
    ref.run(key=4)
    buf = env.empty_graph((T + 1, B), cuda)
    g0 = env.reset(4, n_env=B, out=env._assemble(buf.nodes[0], buf.edges[0], buf.states[0], buf.receivers[0],
                                                 buf.senders[0], None))
    rw, cs = torch.empty_like(ref.rewards), torch.empty_like(ref.costs)
    env.rollout_into(buf, env._obstacles_of(g0), ref.actions, rw, cs, rebuild_first=False)
    torch.cuda.synchronize(cuda)
    for f in ("nodes", "edges", "states", "receivers", "senders"):
        assert torch.equal(getattr(buf, f), getattr(ref.buf, f)), f
    assert torch.equal(rw, ref.rewards) and torch.equal(cs, ref.costs)
