"""Diagnostic: the row predicate and the join on the exact lattice polygons (tests/test_oracle_exact.py),
per grid density, printing every mismatch class (GEOMESA_HIP_LIB picks the library)."""
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, "."); sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from geomesa_amd.join import PolygonIndex, PolygonSet  # noqa: E402
from test_oracle_exact import LATTICE, _locate_exact, lattice_polys  # noqa: E402
import oracle as O  # noqa: E402

polys = lattice_polys()
ps = PolygonSet.from_polygons(polys)
ops = O.OraclePolySet(*ps.to_arrays())
gx, gy = np.meshgrid(LATTICE, LATTICE)
px, py = gx.ravel().copy(), gy.ravel().copy()
exp = np.array([[_locate_exact(parts, float(x), float(y)) for x, y in zip(px, py)] for parts in polys], np.uint8)
ora = np.array([[ops.locate(p, float(x), float(y)) for x, y in zip(px, py)] for p in range(len(polys))], np.uint8)
print("oracle == exact:", np.array_equal(ora, exp), flush=True)
for cells in (0, 64, 16384):
    ix = PolygonIndex(ps, cells_per_poly=cells)
    n = len(px)
    poly = np.repeat(np.arange(len(polys), dtype=np.int32), n)
    loc = ix.relate(poly, np.tile(px, len(polys)), np.tile(py, len(polys))).cpu().numpy().reshape(len(polys), n)
    bad = np.argwhere(loc != exp)
    c = Counter((int(p), int(exp[p, i]), int(loc[p, i])) for p, i in bad)
    print("cells", cells, "relate mismatches", len(bad), dict(c), flush=True)
    for p, i in bad[:8]:
        print("   poly", p, "pt", px[i], py[i], "exp", exp[p, i], "got", loc[p, i])
    pt, pl = ix.join(px, py)
    got = set(zip(pt.cpu().numpy().tolist(), pl.cpu().numpy().tolist()))
    want = {(i, p) for p in range(len(polys)) for i in np.flatnonzero(exp[p] == 2).tolist()}
    print("cells", cells, "join missing", len(want - got), "extra", len(got - want), sorted(want - got)[:5],
          sorted(got - want)[:5], flush=True)
