"""Fused query scan (gm_query_scan): BBOX AND during AND OR-over-polygons of INTERSECTS /
CONTAINS(WITHIN) in one pass, against the oracle (gmo_query_scan: the strict terms plus JTS
PointLocator semantics, pinned by SpatialRelationFunctionsTest's box KATs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def as_np(t):
    return t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)


BOX = "POLYGON((0  0,  0 10, 10 10, 10  0,  0  0))"
SHAPES = [
    "POLYGON((0 0, 0 10, 10 10, 10 0, 0 0), (3 3, 6 3, 6 6, 3 6, 3 3))",
    "MULTIPOLYGON(((20 0, 20 10, 25 10, 25 0, 20 0)), ((25 0, 25 10, 30 10, 30 0, 25 0)))",
    "POLYGON((40 0, 45 10, 50 0, 45 5, 40 0))",
]


def test_query_scan_box_kats_gpu(gpu):  # SpatialRelationFunctionsTest.scala:85-107, 239-262, 359-362
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonSet
    ps = PolygonSet.from_wkt([BOX])
    names = ["int", "edge", "corner", "ext"]
    x = [5.0, 0.0, 0.0, -5.0]
    y = [5.0, 5.0, 0.0, 0.0]
    m, _, _ = F.query_scan(x, y, geoms=ps, op="intersects")
    assert [k for k, v in zip(names, as_np(m)) if v] == ["int", "edge", "corner"]
    m, _, _ = F.query_scan(x, y, geoms=ps, op="contains")
    assert [k for k, v in zip(names, as_np(m)) if v] == ["int"]
    m, _, _ = F.query_scan(x, y, geoms=ps, op="within")
    assert [k for k, v in zip(names, as_np(m)) if v] == ["int"]


def _points(n, seed, ps):
    """Uniform points over the shapes' extent plus every vertex, segment midpoints and points on
    horizontal / vertical lines through vertices (edge and vertex hits for both predicates)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-2, 52, n)
    y = rng.uniform(-2, 12, n)
    x = np.concatenate([x, ps.vx, (ps.vx[1:] + ps.vx[:-1]) / 2, np.full(200, 25.0), np.linspace(-1, 51, 200)])
    y = np.concatenate([y, ps.vy, (ps.vy[1:] + ps.vy[:-1]) / 2, np.linspace(-1, 11, 200), np.full(200, 5.0)])
    t = rng.integers(0, 1000, len(x)).astype(np.int64)
    return x, y, t


@pytest.mark.parametrize("cells", [0, 1, 16, 65536, 1 << 20])   # 1 << 20: a coarse table too large for LDS
@pytest.mark.parametrize("op,oop", [("intersects", 1), ("contains", 2)])
def test_query_scan_parity(gpu, oracle, cells, op, oop):
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonIndex, PolygonSet
    ps = PolygonSet.from_wkt(SHAPES)
    ix = PolygonIndex(ps, cells_per_poly=cells)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    x, y, t = _points(200_000, 3 + cells, ps)
    for bbox, during in [(None, None), ([1, 1, 28, 9], None), (None, (100, 700)), ([-1, -1, 60, 5], (0, 999))]:
        exp = oracle.query_scan(x, y, t, bbox=bbox, during=during, polys=ops, op=oop)
        m, ids, nm = F.query_scan(x, y, t, bbox=bbox, during=during, geoms=ix, op=op, want_ids=True)
        assert np.array_equal(as_np(m), exp), (bbox, during)
        assert nm == int(exp.sum())
        assert np.array_equal(as_np(ids), np.nonzero(exp)[0])


@pytest.mark.parametrize("n", [1, 7, 64, 65, 2049, 100_003])
def test_query_scan_ragged_unaligned(gpu, oracle, n):
    import torch
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonIndex, PolygonSet
    ps = PolygonSet.from_wkt(SHAPES)
    ix = PolygonIndex(ps)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    x, y, t = _points(n + 1, n, ps)
    x, y, t = x[:n + 1], y[:n + 1], t[:n + 1]
    # unaligned device views: offset by one element
    xd = torch.from_numpy(x).cuda()[1:]
    yd = torch.from_numpy(y).cuda()[1:]
    td = torch.from_numpy(t).cuda()[1:]
    exp = oracle.query_scan(x[1:], y[1:], t[1:], bbox=[0, 0, 40, 8], during=(50, 900), polys=ops, op=1)
    m, ids, nm = F.query_scan(xd, yd, td, bbox=[0, 0, 40, 8], during=(50, 900), geoms=ix, op="intersects",
                              want_ids=True)
    assert np.array_equal(as_np(m), exp)
    assert np.array_equal(as_np(ids), np.nonzero(exp)[0])


def test_query_scan_or_of_parts_and_special_values(gpu, oracle):
    """An IDL-split query geometry is an OR of its parts; NaN / inf coordinates never match a
    geometry term; no geometry term = the strict scan."""
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonSet
    ps = PolygonSet.from_wkt(["POLYGON((170 -10, 170 10, 180 10, 180 -10, 170 -10))",
                              "POLYGON((-180 -10, -180 10, -170 10, -170 -10, -180 -10))"])
    ops = oracle.OraclePolySet(*ps.to_arrays())
    rng = np.random.default_rng(4)
    x = rng.uniform(-180, 180, 50_000)
    y = rng.uniform(-20, 20, 50_000)
    x[::17] = np.nan; y[::19] = np.inf; x[::23] = 180.0; x[::29] = -180.0
    for op, oop in (("intersects", 1), ("contains", 2)):
        exp = oracle.query_scan(x, y, polys=ops, op=oop)
        m, _, nm = F.query_scan(x, y, geoms=ps, op=op)
        assert np.array_equal(as_np(m), exp) and nm == int(exp.sum())
    t = np.arange(len(x), dtype=np.int64)
    exp = oracle.strict_scan(x, y, t, [-170, -5, 170, 5], during=(100, 40_000))
    m, _, _ = F.query_scan(x, y, t, bbox=[-170, -5, 170, 5], during=(100, 40_000))
    assert np.array_equal(as_np(m), exp)


def test_query_scan_empty(gpu):
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonSet
    ps = PolygonSet.from_wkt([BOX])
    m, ids, nm = F.query_scan(np.zeros(0), np.zeros(0), geoms=ps, want_ids=True)
    assert nm == 0 and m.numel() == 0


@pytest.mark.parametrize("cells", [4096, 65536])
def test_query_scan_lobed_polygon_near_edges(gpu, oracle, cells):
    """The bench's query geometry (1,024-vertex lobed ring with a 64-vertex hole) over points in its
    envelope plus every vertex, every edge midpoint and points a hair off each vertex: the scan's lookup
    chain (coarse sub-block masks, fine words with boundary shortcuts, line entries, compact and generic
    blobs walked by the block) against the oracle's PointLocator, both predicates."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonIndex
    ps = bench.query_polygon()
    ix = PolygonIndex(ps, cells_per_poly=cells)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    rng = np.random.default_rng(cells)
    x = [rng.uniform(-15, 35, 400_000)]
    y = [rng.uniform(30, 64, 400_000)]
    vx, vy = ps.vx, ps.vy
    x += [vx, (vx[1:] + vx[:-1]) / 2]
    y += [vy, (vy[1:] + vy[:-1]) / 2]
    for eps in (1e-12, 1e-9, 1e-6, 1e-3):
        for sx, sy in ((1, 0), (0, 1), (-1, -1), (1, -1)):
            x.append(vx + sx * eps)
            y.append(vy + sy * eps)
    x, y = np.concatenate(x), np.concatenate(y)
    for op, oop in (("intersects", 1), ("contains", 2)):
        exp = oracle.query_scan(x, y, polys=ops, op=oop)
        m, ids, nm = F.query_scan(x, y, geoms=ix, op=op, want_ids=True)
        assert np.array_equal(as_np(m), exp), op
        assert nm == int(exp.sum()) and np.array_equal(as_np(ids), np.nonzero(exp)[0])


@pytest.mark.parametrize("which", ["lattice", "stacked"])
@pytest.mark.parametrize("cells", [0, 16, 65536])
def test_query_scan_lattice_exact(gpu, oracle, cells, which):
    """The fused filter's polygon term against exact rational arithmetic (tests/test_oracle_exact.py):
    overlapping lattice polygons with holes and MultiPolygon parts sharing an edge / a vertex, every
    point of a 1/8 lattice (thousands exactly on edges).  The polygon term is the OR of the set's
    polygons: contains = INTERIOR of some polygon, intersects = not EXTERIOR of some polygon."""
    from geomesa_amd import filters as F
    from geomesa_amd.join import PolygonIndex, PolygonSet
    from test_oracle_exact import exact_lattice
    polys, x, y, loc = exact_lattice(which)
    ps = PolygonSet.from_polygons(polys)
    t = np.arange(len(x), dtype=np.int64)
    ix = PolygonIndex(ps, cells_per_poly=cells)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    for op, oop, exp in (("contains", 2, (loc == 2).any(0)), ("intersects", 1, (loc != 0).any(0))):
        assert np.array_equal(oracle.query_scan(x, y, t, polys=ops, op=oop), exp)
        m, ids, nm = F.query_scan(x, y, t, bbox=[-0.5, -0.5, 6.5, 6.5], during=(0, len(x)), geoms=ix, op=op,
                                  want_ids=True)
        assert np.array_equal(as_np(m), exp), (op, np.flatnonzero(as_np(m) != exp)[:10])
        assert nm == int(exp.sum())
