"""Times gm_z3_histogram over 1B resident points for several histogram lengths (occupancy probe)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from geomesa_amd import _lib  # noqa: E402
from bench import gen_points  # noqa: E402

N = 1_000_000_000
ctx = _lib.context()
x = torch.empty(N, dtype=torch.float64, device="cuda"); y = torch.empty_like(x)
t = torch.empty(N, dtype=torch.int64, device="cuda")
gen_points(ctx, N, 0, (-180.0, -90.0, 180.0, 90.0), x, y, t)
P = _lib.ptr
res = {}
for L in (16, 64, 256, 512, 1024, 2048):
    c = torch.zeros((54, L), dtype=torch.int64, device="cuda")
    p = torch.zeros(54, dtype=torch.uint8, device="cuda")
    tl = torch.zeros(2, dtype=torch.int64, device="cuda")
    f = lambda: _lib.check(ctx.lib.gm_z3_histogram(ctx.handle, P(x), P(y), P(t), N, 1, L, 0, 2608, 54, P(p), P(c),
                                                   P(tl)), "hist")
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        f()
    e1.record(); torch.cuda.synchronize()
    res[L] = e0.elapsed_time(e1) / 5
    print(L, res[L], flush=True)
print(json.dumps(res))
