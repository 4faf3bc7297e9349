"""torch.ops.dgppo custom ops (dgppo_fov_amd/ops.py): registration, fake (meta) kernels, the no-CPU
rule, and on the GPU bit-identity with the raw C-ABI call and CUDA-graph capture."""
import ctypes

import numpy as np
import pytest
import torch

from dgppo_fov_amd import _lib, ops  # noqa: F401  (registers torch.ops.dgppo.*)

OPS = ("env_reset", "env_step", "gnn_attn_fwd", "gnn_attn_bwd", "gae", "grad_norm", "adam")


def test_ops_registered_with_schemas():
    for name in OPS:
        op = getattr(torch.ops.dgppo, name)
        schema = str(op.default._schema)
        assert schema.startswith(f"dgppo::{name}("), schema
        assert schema.endswith("-> ()"), schema  # every op writes caller-owned outputs in place
    # mutated outputs are declared as such (aliasing annotations "(a!)")
    import re

    assert re.search(r"Tensor\(a\d+!\) nodes", str(torch.ops.dgppo.env_step.default._schema))
    assert re.search(r"Tensor\(a\d+!\) param", str(torch.ops.dgppo.adam.default._schema))
    assert re.search(r"Tensor states,", str(torch.ops.dgppo.env_step.default._schema))  # inputs are read-only


def test_fake_kernels_trace_without_a_device():
    from torch._subclasses.fake_tensor import FakeTensorMode

    with FakeTensorMode():
        B, T, n, nh = 2, 5, 3, 2
        hs = torch.empty(B, T, n, nh)
        l = torch.empty(B, T)
        Vh, Vl = torch.empty(B, T + 1, n, nh), torch.empty(B, T + 1)
        Qh, Ql = torch.empty(B, T, n, nh), torch.empty(B, T)
        torch.ops.dgppo.gae(hs, l, Vh, Vl, Qh, Ql, 0.99, 0.95)
        p, g, m, v, st = (torch.empty(7) for _ in range(5))
        torch.ops.dgppo.adam(p, g, m, v, st, 1e-3, 0.9, 0.999, 1e-8, 2.0)
        torch.ops.dgppo.grad_norm(g, st)


def test_ops_refuse_cpu_tensors():
    p = torch.zeros(4)
    with pytest.raises(_lib.NativeLibraryError):
        torch.ops.dgppo.grad_norm(p, torch.zeros(3))
    with pytest.raises(_lib.NativeLibraryError):
        torch.ops.dgppo.adam(p, p, p.clone(), p.clone(), torch.zeros(3), 1e-3, 0.9, 0.999, 1e-8, 2.0)


def _raw_env_step(env, g, action, out, reward, cost):
    """The same step through the C-ABI directly (ctypes), bypassing the torch op."""
    io = _lib.EnvStepIO()
    io.states, io.states_stride = g.states.data_ptr(), ops._stride(g.states, 2)
    ob = env._obstacles_of(g)
    io.obstacles, io.obstacles_stride = ob.data_ptr(), ob.stride(-3)
    io.action, io.action_stride = action.data_ptr(), ops._stride(action, 2)
    io.ray_dirs = env._ray_table(g.states.device).data_ptr()
    io.nodes, io.nodes_stride = out.nodes.data_ptr(), ops._stride(out.nodes, 2)
    io.edges, io.edges_stride = out.edges.data_ptr(), ops._stride(out.edges, 2)
    io.out_states, io.out_states_stride = out.states.data_ptr(), ops._stride(out.states, 2)
    io.receivers, io.senders = out.receivers.data_ptr(), out.senders.data_ptr()
    io.edge_index_stride = ops._stride(out.receivers, 1)
    io.reward, io.reward_stride = reward.data_ptr(), 1
    io.cost, io.cost_stride = cost.data_ptr(), ops._stride(cost, 2)
    io.n_env = g.states.shape[0]
    _lib.check(_lib.load().dgppo_env_step(ctypes.byref(env.cfg), ctypes.byref(io),
                                          _lib.stream_handle(g.states.device)), "dgppo_env_step")


@pytest.mark.gpu
def test_env_step_op_matches_c_abi_and_captures(cuda):
    from dgppo_fov_amd.env import make_env

    env = make_env("LidarSpread", 8, num_obs=3, device=cuda)
    B = 512
    g = env.reset(key=3, n_env=B)
    a = torch.rand((B, 8, 2), device=cuda) * 2 - 1
    outs = []
    for path in ("op", "raw", "graph"):
        out = env.empty_graph((B,), cuda)
        r = torch.empty(B, device=cuda)
        c = torch.empty((B, 8, 2), device=cuda)
        if path == "op":
            torch.ops.dgppo.env_step(env._cfg_handle, g.states, env._obstacles_of(g), a, env._ray_table(cuda), out.nodes, out.edges,
                                     out.states, out.receivers, out.senders, r, c)
        elif path == "raw":
            _raw_env_step(env, g, a, out, r, c)
        else:
            torch.cuda.synchronize()
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg):
                env.step_into(g, a, out, r, c)  # MultiAgentEnv.step_into -> torch.ops.dgppo.env_step
            for t in (out.nodes, out.edges, r):
                t.fill_(float("nan"))
            cg.replay()
        torch.cuda.synchronize()
        outs.append([x.cpu().numpy() for x in (out.nodes, out.edges, out.states, out.receivers, out.senders, r, c)])
    for other in outs[1:]:
        for x, y in zip(outs[0], other):
            assert np.array_equal(x, y)


@pytest.mark.gpu
def test_opcheck_schema_and_fake(cuda):
    """torch.library.opcheck: declared mutations match what the kernels write, fake kernels agree."""
    B, T, n, nh = 3, 16, 4, 2
    hs = torch.randn(B, T, n, nh, device=cuda)
    l = torch.randn(B, T, device=cuda)
    Vh, Vl = torch.randn(B, T + 1, n, nh, device=cuda), torch.randn(B, T + 1, device=cuda)
    Qh, Ql = torch.empty(B, T, n, nh, device=cuda), torch.empty(B, T, device=cuda)
    utils = ("test_schema", "test_faketensor")
    torch.library.opcheck(torch.ops.dgppo.gae.default, (hs, l, Vh, Vl, Qh, Ql, 0.99, 0.95), test_utils=utils)
    p, g = torch.randn(1000, device=cuda), torch.randn(1000, device=cuda)
    m, v, st = torch.zeros_like(p), torch.zeros_like(p), torch.zeros(3, device=cuda)
    torch.library.opcheck(torch.ops.dgppo.grad_norm.default, (g, st), test_utils=utils)
    torch.library.opcheck(torch.ops.dgppo.adam.default, (p, g, m, v, st, 1e-3, 0.9, 0.999, 1e-8, 2.0),
                          test_utils=utils)
