"""HBM write roofline probe: torch fill_ (coalesced 16-byte stores) and copy_ over buffers the size of one
persistent rollout's output (4.6 GB), HIP events, median of 10."""
import json

import torch


def timeit(fn, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


n = 4_643_094_528 // 4
a = torch.empty(n, device="cuda")
b = torch.empty(n, device="cuda")
t_fill = timeit(lambda: a.fill_(1.0))
t_copy = timeit(lambda: b.copy_(a))
print(json.dumps({"bytes": n * 4, "fill_ms": t_fill, "fill_TBs": n * 4 / t_fill / 1e9,
                  "copy_ms": t_copy, "copy_TBs_rw": 2 * n * 4 / t_copy / 1e9}))
