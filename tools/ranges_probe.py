"""Times the batched XZ2 / Z3 ranges entry points on the bench's query sets (for rocprofv3 runs)."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from geomesa_amd import _lib  # noqa: E402
from geomesa_amd import ranges as R  # noqa: E402


def main(nq=100_000):
    ctx = _lib.context()
    rng = np.random.default_rng(2)
    wq = 10 ** rng.uniform(-2, np.log10(20), (nq, 2)) / 2
    cq = np.stack([rng.uniform(-180 + wq[:, 0], 180 - wq[:, 0]), rng.uniform(-90 + wq[:, 1], 90 - wq[:, 1])], 1)
    win = np.ascontiguousarray(np.concatenate([cq - wq, cq + wq], 1).reshape(-1))
    woff = np.arange(nq + 1, dtype=np.int32)
    args = (ctx.handle, nq, woff.ctypes.data, win.ctypes.data, 12, 2000)
    for k in range(3):
        t0 = time.time()
        offs, rr, _ = R.call_raw(ctx.lib.gm_xz2_ranges, args, nq, nq * 256)
        print("xz2 ranges: %d queries, %d ranges, %.1f ms" % (nq, int(offs[-1]), (time.time() - t0) * 1e3), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100_000)


def pinned_variant(nq=100_000):
    """Same calls with a reused pinned host output buffer (isolates pageable-memory effects)."""
    import ctypes
    import torch
    ctx = _lib.context()
    rng = np.random.default_rng(2)
    wq = 10 ** rng.uniform(-2, np.log10(20), (nq, 2)) / 2
    cq = np.stack([rng.uniform(-180 + wq[:, 0], 180 - wq[:, 0]), rng.uniform(-90 + wq[:, 1], 90 - wq[:, 1])], 1)
    win = np.ascontiguousarray(np.concatenate([cq - wq, cq + wq], 1).reshape(-1))
    woff = np.arange(nq + 1, dtype=np.int32)
    cap = 12_000_000
    buf = torch.empty(cap * 24, dtype=torch.uint8, pin_memory=True)
    out_off = np.zeros(nq + 1, np.int64)
    qst = np.zeros(nq, np.int32)
    needed = ctypes.c_int64()
    for k in range(4):
        t0 = time.time()
        rc = ctx.lib.gm_xz2_ranges(ctx.handle, nq, woff.ctypes.data, win.ctypes.data, 12, 2000, out_off.ctypes.data,
                                   ctypes.c_void_p(buf.data_ptr()), cap, ctypes.byref(needed), qst.ctypes.data)
        print("pinned xz2 ranges rc=%d: %d ranges, %.1f ms" % (rc, needed.value, (time.time() - t0) * 1e3), flush=True)


if __name__ == "__main__" and len(sys.argv) > 2:
    pinned_variant()
