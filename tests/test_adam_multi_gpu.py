"""dgppo_adam_multi (ABI 12: the clip + finite check + Adam steps of several nets in two launches) against the
per-net dgppo_grad_norm + dgppo_adam pair it replaces in DGPPO._mb_apply: parameters, moments and state
bit-identical over several steps, including a step one net skips (non-finite gradient, optax.apply_if_finite) and
nets of different sizes, learning rates and clip norms."""
import pytest
import torch

from dgppo_fov_amd.nn import kernels as K

pytestmark = pytest.mark.gpu


def _nets(cuda, sizes, seed):
    g = torch.Generator(device=cuda).manual_seed(seed)
    out = []
    for i, n in enumerate(sizes):
        p = torch.randn(n, device=cuda, generator=g)
        out.append(dict(param=p, m=torch.zeros_like(p), v=torch.zeros_like(p),
                        state=torch.zeros(3, device=cuda), lr=[1e-3, 3e-4, 1e-3, 5e-4][i], max_norm=[2.0, 2.0, 0.5, 1.0][i]))
    return out


def _clone(nets):
    return [{k: (v.clone() if torch.is_tensor(v) else v) for k, v in d.items()} for d in nets]


@pytest.mark.parametrize("sizes", [(52_000, 37_000, 61_000), (1, 300, 2_500_000, 70_000)])
def test_adam_multi_matches_per_net_pairs(cuda, sizes):
    a = _nets(cuda, sizes, 0)
    b = _clone(a)
    g = torch.Generator(device=cuda).manual_seed(1)
    for step in range(4):
        grads = [torch.randn(n, device=cuda, generator=g) * (0.01 if step % 2 else 3.0) for n in sizes]
        if step == 2:
            grads[1][len(grads[1]) // 2] = float("inf")  # net 1 skips this step; the others apply theirs
        for d, gr in zip(a, grads):
            K.grad_norm(gr, d["state"])
            K.adam(d["param"], gr, d["m"], d["v"], d["state"], d["lr"], max_norm=d["max_norm"])
        K.adam_multi([(d["param"], gr, d["m"], d["v"], d["state"], d["lr"], d["max_norm"]) for d, gr in zip(b, grads)])
        torch.cuda.synchronize()
        for k, (x, y) in enumerate(zip(a, b)):
            for f in ("param", "m", "v", "state"):
                assert torch.equal(x[f], y[f]), f"step {step} net {k} {f}"
    assert a[1]["state"][2].item() == 3.0 and a[0]["state"][2].item() == 4.0  # the skipped step is not counted
