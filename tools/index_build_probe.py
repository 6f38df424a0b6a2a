"""Times PolygonIndex construction (host build + upload) for the bench's 3,200 synthetic counties and
the US states, with GM_PIP_DEBUG phase timings on stderr.  Usage: python tools/index_build_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
os.environ.setdefault("GM_PIP_DEBUG", "1")

import torch  # noqa: E402
from geomesa_amd import _lib  # noqa: E402
from geomesa_amd.join import PolygonIndex, synthetic_counties  # noqa: E402

ctx = _lib.context(0)
ps = synthetic_counties(80, 40)
for cpp in (8192, 0):
    for rep in range(2):
        t0 = time.time()
        ix = PolygonIndex(ps, ctx, cpp)
        torch.cuda.synchronize()
        print("counties cells_per_poly=%d: %.3f s  %s" % (cpp, time.time() - t0, ix.stats()), flush=True)
        del ix
from shapefile import us_states  # noqa: E402
st, _ = us_states()
t0 = time.time()
ix = PolygonIndex(st, ctx)
torch.cuda.synchronize()
print("states: %.3f s %s" % (time.time() - t0, ix.stats()), flush=True)
