"""Times gm_sort_keys on the bench's table leg (250M rows of Z3 keys of uniform points over 2020,
53 week bins, optionally with a 4-way shard byte) and checks the result on the GPU: keys in table order,
perm a permutation that maps the output back to the input.  For A/B runs of library builds
(GEOMESA_HIP_LIB) in one GPU call.

    python tools/sort_probe.py [rows] [sharded]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from geomesa_amd import _lib  # noqa: E402
from geomesa_amd.curve import Z3SFC  # noqa: E402


def main(n=250_000_000, sharded=False):
    ctx = _lib.context()
    dev = torch.device("cuda", ctx.device)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.rand(n, device=dev, generator=g, dtype=torch.float64) * 360 - 180
    y = torch.rand(n, device=dev, generator=g, dtype=torch.float64) * 180 - 90
    t = (torch.rand(n, device=dev, generator=g, dtype=torch.float64) * 31622400000).to(torch.int64) + 1577836800000
    b, z = Z3SFC("week").index_keys(x, y, t)
    del x, y, t
    sh = (torch.arange(n, device=dev) % 4).to(torch.uint8) if sharded else None
    ob, oz = torch.empty_like(b), torch.empty_like(z)
    osh = torch.empty_like(sh) if sharded else None
    perm = torch.empty(n, dtype=torch.int64, device=dev)
    P = _lib.ptr

    def run():
        _lib.check(ctx.lib.gm_sort_keys(ctx.handle, P(sh), P(b), P(z), n, P(osh), P(ob), P(oz), P(perm)), "gm_sort_keys")
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    if os.environ.get("GM_SORT_PROBE_NOCHECK"):   # timing-only library variants write partial output
        print("sort %d rows: best %.2f ms, mean %.2f ms, unchecked" % (n, min(ts), sum(ts) / len(ts)), flush=True)
        return
    # checks: output = input[perm], keys nondecreasing in (shard, bin unsigned, z unsigned) order
    ok = bool(torch.equal(ob, b[perm])) and bool(torch.equal(oz, z[perm]))
    hi = (ob.to(torch.int64) & 0xffff) | ((osh.to(torch.int64) << 16) if sharded else 0)
    lo = oz ^ (-(1 << 63))
    dh, dl = hi[1:] - hi[:-1], lo[1:] >= lo[:-1]
    ok = ok and bool(((dh > 0) | ((dh == 0) & dl)).all())
    ok = ok and bool(torch.equal(torch.sort(perm).values, torch.arange(n, device=dev)))
    if sharded:
        ok = ok and bool(torch.equal(osh, sh[perm]))
    print("sort %d rows%s: best %.2f ms, mean %.2f ms, ok=%s" % (n, " sharded" if sharded else "", min(ts),
                                                               sum(ts) / len(ts), ok), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 250_000_000, len(sys.argv) > 2 and sys.argv[2] == "1")
