"""Times gm_xz2_index / gm_xz3_index over 100M envelopes shaped as the bench's configs[4] leg (tuning
probe; GEOMESA_HIP_LIB selects a variant)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from geomesa_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    ctx = _lib.context()
    lib, h, P = ctx.lib, ctx.handle, _lib.ptr
    x = torch.empty(n, dtype=torch.float64, device="cuda"); y = torch.empty_like(x)
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    bench.gen_points(ctx, n, 0, (-180.0, -90.0, 180.0, 90.0), x, y, t)
    g = torch.Generator(device="cuda").manual_seed(11)
    w = torch.pow(10.0, torch.rand(n, device="cuda", dtype=torch.float64, generator=g) * 7 - 6)
    hg = torch.pow(10.0, torch.rand(n, device="cuda", dtype=torch.float64, generator=g) * 7 - 6)
    xmax = torch.clamp(x + w, max=180.0); ymax = torch.clamp(y + hg, max=90.0)
    zmin = torch.remainder(t, 604_800_000).to(torch.float64) / 1000.0
    zmax = torch.clamp(zmin + torch.pow(10.0, torch.rand(n, device="cuda", dtype=torch.float64, generator=g) * 4.94),
                       max=604800.0)
    del w, hg, t
    xo = torch.empty(n, dtype=torch.int64, device="cuda")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, fn, bpu in (("xz2_index", lambda: lib.gm_xz2_index(h, P(x), P(y), P(xmax), P(ymax), n, 12, 0, P(xo), None, None), 40),
                          ("xz3_index", lambda: lib.gm_xz3_index(h, P(x), P(y), P(zmin), P(xmax), P(ymax), P(zmax), n, 12, 1, 0,
                                                                 P(xo), None, None), 56)):
        fn(); torch.cuda.synchronize()
        ev0.record()
        for _ in range(10):
            assert fn() == 0
        ev1.record(); torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / 10
        print("%-10s %8.4f ms  %6.3f of 8 TB/s" % (name, ms, bpu * n / ms / 1e9 / 8.0), flush=True)


if __name__ == "__main__":
    main()
