"""Per-phase cycle sums of k_xzranges from a GM_XR_STAMPS build (timing experiment):
GEOMESA_HIP_LIB=geomesa_amd/lib/xr_stamps.so python tools/xr_phases.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from geomesa_amd import _lib  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import ranges_probe as RP  # noqa: E402

ctx = _lib.context()
lib = ctx.lib
ph = (ctypes.c_ulonglong * 8)()
nq = 100_000
win, win3 = RP.windows(nq)
woff = np.arange(nq + 1, dtype=np.int32)
for name, fn, args in (("xz2", lib.gm_xz2_ranges, (ctx.handle, nq, woff.ctypes.data, win.ctypes.data, 12, 2000)),
                       ("xz3", lib.gm_xz3_ranges, (ctx.handle, nq, woff.ctypes.data, win3.ctypes.data, 12, 1, 2000))):
    RP.timed_dev(name, fn, args, nq, nq * 1024, reps=1)
    lib.gm_debug_xr_phases(ph, 1)
    RP.timed_dev(name, fn, args, nq, nq * 1024, reps=1)
    lib.gm_debug_xr_phases(ph, 1)
    names = ["walk", "bottom-out", "sort_merge", "batch_finish", "-", "runs", "rank", "merge"]
    tot = sum(ph[k] for k in range(4))
    print(name, " ".join("%s %.1f%%" % (names[k], 100.0 * ph[k] / tot) for k in (0, 1, 2, 3, 5, 6, 7)), flush=True)
