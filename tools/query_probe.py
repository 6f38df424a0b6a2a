"""Times gm_query_scan on 1B resident points (tuning probe; GEOMESA_HIP_LIB selects a variant).

Cases: the bench's BBOX + DURING + INTERSECTS query and INTERSECTS alone over world-uniform points,
and INTERSECTS / CONTAINS over points drawn inside the query polygon's envelope (dense: most rows
reach the cell lookup and ~60% match)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from geomesa_amd import _lib  # noqa: E402
from geomesa_amd.join import PolygonIndex  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    cells = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    ctx = _lib.context()
    lib, h, P = ctx.lib, ctx.handle, _lib.ptr
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    mask = torch.empty((n + 63) // 64, dtype=torch.int64, device="cuda")
    ix = PolygonIndex(bench.query_polygon(), cells_per_poly=cells)
    bb = (ctypes.c_double * 4)(-10.0, 35.0, 30.0, 60.0)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timeit(name, fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ev0.record()
        for _ in range(reps):
            rc = fn()
            assert rc == 0, rc
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / reps
        nm = ctypes.c_int64()
        fn(ctypes.byref(nm))
        print("%-28s %8.3f ms  %6.1f G rows/s  matches %d" % (name, ms, n / ms / 1e6, nm.value), flush=True)

    for region, bounds in (("world", (-180.0, -90.0, 180.0, 90.0)), ("envelope", (-12.0, 35.0, 32.0, 59.0))):
        bench.gen_points(ctx, n, 0, bounds, x, y, t)
        timeit(region + " bbox+during+intersects",
               lambda nm=None: lib.gm_query_scan(h, P(x), P(y), P(t), n, bb, 1, 1590969600000, 1591617600000, ix._h, 1,
                                                 P(mask), None, 0, nm))
        timeit(region + " intersects",
               lambda nm=None: lib.gm_query_scan(h, P(x), P(y), None, n, None, 0, 0, 0, ix._h, 1, P(mask), None, 0, nm))
        timeit(region + " contains",
               lambda nm=None: lib.gm_query_scan(h, P(x), P(y), None, n, None, 0, 0, 0, ix._h, 2, P(mask), None, 0, nm))
        timeit(region + " bbox+during (no geometry)",
               lambda nm=None: lib.gm_query_scan(h, P(x), P(y), P(t), n, bb, 1, 1590969600000, 1591617600000, None, 0,
                                                 P(mask), None, 0, nm))


if __name__ == "__main__":
    main()
