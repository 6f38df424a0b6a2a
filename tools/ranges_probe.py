"""Times the batched XZ2 / XZ3 / Z3 ranges entry points on the bench's query sets and prints a digest
of each result (so two library builds, picked with GEOMESA_HIP_LIB, can be compared in one GPU call).

    python tools/ranges_probe.py [n_queries]
"""
import ctypes
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from geomesa_amd import _lib  # noqa: E402
from geomesa_amd import ranges as R  # noqa: E402


def windows(nq, seed=2):
    rng = np.random.default_rng(seed)
    wq = 10 ** rng.uniform(-2, np.log10(20), (nq, 2)) / 2
    cq = np.stack([rng.uniform(-180 + wq[:, 0], 180 - wq[:, 0]), rng.uniform(-90 + wq[:, 1], 90 - wq[:, 1])], 1)
    win = np.ascontiguousarray(np.concatenate([cq - wq, cq + wq], 1))
    tw0 = rng.uniform(0, 604800 - 172800, nq)
    tw1 = tw0 + 10 ** rng.uniform(np.log10(60), np.log10(172800), nq)
    win3 = np.ascontiguousarray(np.stack([win[:, 0], win[:, 1], tw0, win[:, 2], win[:, 3], tw1], 1))
    return win.reshape(-1), win3.reshape(-1)


def timed(name, fn, args, nq, reps=3):
    offs, rr, qst = R.call_raw(fn, args, nq, nq * 256, pinned=True)
    cap = int(offs[-1]) + 1024
    ts = []
    for _ in range(reps):
        t0 = time.time()
        offs, rr, qst = R.call_raw(fn, args, nq, cap, pinned=True)
        ts.append((time.time() - t0) * 1e3)
    n = int(offs[-1])
    dig = hashlib.sha1(offs.tobytes() + np.asarray(rr[:n]).tobytes() + qst.tobytes()).hexdigest()[:12]
    print("%-4s %d queries %10d ranges  best %8.2f ms  mean %8.2f ms  digest %s"
          % (name, nq, n, min(ts), sum(ts) / len(ts), dig), flush=True)


def timed_dev(name, fn, args, nq, cap, reps=3):
    """The same entry point writing into device memory (the ranges stay in HBM for a device-side
    consumer such as gm_key_range_scan): no copy back; the digest must equal the host-output run's."""
    import torch
    out = torch.empty(int(cap) * R.RANGE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    ts = []
    for _ in range(reps + 1):
        offs = np.zeros(nq + 1, np.int64)
        needed = ctypes.c_int64()
        qst = np.zeros(nq, np.int32)
        torch.cuda.synchronize()
        t0 = time.time()
        _lib.check(fn(*args, offs.ctypes.data, out.data_ptr(), int(cap), ctypes.byref(needed), qst.ctypes.data), name)
        torch.cuda.synchronize()
        ts.append((time.time() - t0) * 1e3)
    ts = ts[1:]
    n = int(offs[-1])
    rr = out[:n * R.RANGE_DTYPE.itemsize].cpu().numpy().view(R.RANGE_DTYPE)
    dig = hashlib.sha1(offs.tobytes() + np.asarray(rr[:n]).tobytes() + qst.tobytes()).hexdigest()[:12]
    print("%-4s %d queries %10d ranges  best %8.2f ms  mean %8.2f ms  digest %s  (device output)"
          % (name, nq, n, min(ts), sum(ts) / len(ts), dig), flush=True)


def main(nq=100_000):
    ctx = _lib.context()
    if os.environ.get("GM_RANGES_CHUNK"):   # pipelined chunk size (GM_PARAM_RANGES_CHUNK) for sweeps
        ctx.set_param(_lib.GM_PARAM_RANGES_CHUNK, int(os.environ["GM_RANGES_CHUNK"]))
    lib, h = ctx.lib, ctx.handle
    win, win3 = windows(nq)
    woff = np.arange(nq + 1, dtype=np.int32)
    timed("xz2", lib.gm_xz2_ranges, (h, nq, woff.ctypes.data, win.ctypes.data, 12, 2000), nq)
    timed("xz3", lib.gm_xz3_ranges, (h, nq, woff.ctypes.data, win3.ctypes.data, 12, 1, 2000), nq)
    if os.environ.get("GM_RANGES_DEV", "1") == "1":
        timed_dev("xz2", lib.gm_xz2_ranges, (h, nq, woff.ctypes.data, win.ctypes.data, 12, 2000), nq, nq * 256)
        timed_dev("xz3", lib.gm_xz3_ranges, (h, nq, woff.ctypes.data, win3.ctypes.data, 12, 1, 2000), nq, nq * 1024)
    rng = np.random.default_rng(1)
    qs = []
    for _ in range(4096):
        w = 10 ** rng.uniform(-1, 1); hh = 10 ** rng.uniform(-1, 1)
        cx = rng.uniform(-170, 170); cy = rng.uniform(-80, 80); t0 = int(rng.integers(0, 500000))
        qs.append(([(cx - w, cy - hh, cx + w, cy + hh)], [(t0, t0 + 86400)]))
    from geomesa_amd.curve import Z3SFC
    fn, args, n3, _ = R.prepare_z3(Z3SFC("week"), qs, 64, 2000)
    timed("z3", fn, args, n3)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 100_000)
