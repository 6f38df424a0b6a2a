"""Times PolygonIndex construction (device build, then the host build) for the bench's 3,200 synthetic counties and
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
for mode in (0, 1):   # GM_PARAM_INDEX_BUILD: device, host
    ctx.set_param(_lib.GM_PARAM_INDEX_BUILD, mode)
    for rep in range(3):
        t0 = time.time()
        ix = PolygonIndex(ps, ctx, 0)
        torch.cuda.synchronize()
        print("counties %s build: %.3f s  %s" % ("device" if mode == 0 else "host", time.time() - t0, ix.stats()),
              flush=True)
        del ix
ctx.set_param(_lib.GM_PARAM_INDEX_BUILD, 0)
from shapefile import us_states  # noqa: E402
st, _ = us_states()
t0 = time.time()
ix = PolygonIndex(st, ctx)
torch.cuda.synchronize()
print("states: %.3f s %s" % (time.time() - t0, ix.stats()), flush=True)
