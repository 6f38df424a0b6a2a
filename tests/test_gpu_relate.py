"""GPU parity for the row-wise predicate path (Spark SQL st_* UDFs without the join rule):
gm_pip_relate's per-row location against the oracle's PointLocator restatement (oracle gmo_locate),
including points exactly on vertices and edges, holes, multipolygon parts and null rows; and the
kernels against exact rational arithmetic on lattice polygons (tests/test_oracle_exact.py), which pins
the boundary cases the reference's box KATs leave open."""
import contextlib

import numpy as np
import pytest

from test_gpu_parity import as_np

pytestmark = pytest.mark.gpu

NX, NY = 16, 8


def rows(ps, n, seed):
    from geomesa_amd.join import CONUS, synthetic_points
    rng = np.random.default_rng(seed)
    px, py = synthetic_points(n, seed=seed)
    # the polygon of the point's grid cell, a neighbour, or a random one
    x0, y0, x1, y1 = CONUS
    i = np.clip(((px - x0) / (x1 - x0) * NX).astype(int), 0, NX - 1)
    j = np.clip(((py - y0) / (y1 - y0) * NY).astype(int), 0, NY - 1)
    own = j * NX + i
    pick = rng.uniform(size=n)
    poly = np.where(pick < 0.7, own, np.where(pick < 0.85, np.clip(own + rng.integers(-1, 2, n), 0, NX * NY - 1),
                                             rng.integers(0, NX * NY, n)))
    # vertices (boundary) and edge midpoints of the row's polygon
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    k = rng.integers(0, n, n // 10)
    for r in k:
        p = poly[r]
        v = rng.integers(rvo[pro[ppo[p]]], rvo[pro[ppo[p + 1]]])
        if rng.uniform() < 0.5 or v + 1 >= len(vx):
            px[r], py[r] = vx[v], vy[v]
        else:
            px[r], py[r] = 0.5 * (vx[v] + vx[v + 1]), 0.5 * (vy[v] + vy[v + 1])
    poly = poly.astype(np.int32)
    poly[rng.uniform(size=n) < 0.02] = -1   # null rows
    px[::997] = np.nan
    return poly, px, py


@contextlib.contextmanager
def rows64(on):
    """GM_PARAM_RELATE_ROWS64: the kernel with 64-bit queue rows and the join's bitmap (the path of
    calls with 2^32 rows or more) instead of the default 32-bit rows and the finer bitmap."""
    from geomesa_amd import _lib
    ctx = _lib.context()
    ctx.set_param(_lib.GM_PARAM_RELATE_ROWS64, 1 if on else 0)
    try:
        yield
    finally:
        ctx.set_param(_lib.GM_PARAM_RELATE_ROWS64, 0)


@pytest.mark.parametrize("wide", [False, True])
@pytest.mark.parametrize("cells", [0, 64, 16384])
def test_relate_rows_match_oracle(gpu, oracle, cells, wide):
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(NX, NY)
    poly, px, py = rows(ps, 60_000, seed=3 + cells)
    ix = PolygonIndex(ps, cells_per_poly=cells)
    with rows64(wide):
        loc = as_np(ix.relate(poly, px, py))
    ops = oracle.OraclePolySet(*ps.to_arrays())
    exp = np.array([255 if p < 0 else ops.locate(int(p), x, y) for p, x, y in zip(poly, px, py)], np.uint8)
    assert np.array_equal(loc, exp), np.flatnonzero(loc != exp)[:10]
    assert (exp == 1).sum() > 1000 and (exp == 2).sum() > 1000   # boundary and interior both exercised


def test_row_predicates(gpu, oracle):
    import torch
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(NX, NY)
    poly, px, py = rows(ps, 20_000, seed=11)
    ix = PolygonIndex(ps)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    valid = poly >= 0
    con, null = ix.predicate("st_contains", poly, px, py)
    assert np.array_equal(as_np(null), ~valid)
    exp = np.array([p >= 0 and ops.contains(int(p), x, y) for p, x, y in zip(poly, px, py)])
    assert np.array_equal(as_np(con), exp)
    it, _ = ix.predicate("st_intersects", poly, px, py)
    exp = np.array([p >= 0 and ops.intersects(int(p), x, y) for p, x, y in zip(poly, px, py)])
    assert np.array_equal(as_np(it), exp)
    dis, _ = ix.predicate("st_disjoint", poly, px, py)
    assert np.array_equal(as_np(dis)[valid], ~exp[valid])
    tou, _ = ix.predicate("st_touches", poly, px, py)
    cov, _ = ix.predicate("st_covers", poly, px, py)
    assert torch.equal(cov, it) and np.array_equal(as_np(tou), as_np(it) & ~as_np(con))
    cr, _ = ix.predicate("st_crosses", poly, px, py)
    assert not as_np(cr).any()


def test_relate_box_kats(gpu):
    """SpatialRelationFunctionsTest.scala:85-112 box cases, row-wise: interior true; edge, corner and
    exterior false for st_contains; the edge and corner are st_intersects / st_touches."""
    from geomesa_amd.join import PolygonIndex, PolygonSet
    ps = PolygonSet.from_polygons([[[[(0, 0), (2, 0), (2, 2), (0, 2)]]], [[[(10, 10), (12, 10), (12, 12), (10, 12)]]]])
    ix = PolygonIndex(ps)
    px = [1.0, 2.0, 0.0, 3.0, 1.0, 11.0, 1.0]
    py = [1.0, 1.0, 0.0, 1.0, 1.0, 11.0, 1.0]
    poly = [0, 0, 0, 0, 1, 1, -1]
    assert as_np(ix.relate(poly, px, py)).tolist() == [2, 1, 1, 0, 0, 2, 255]
    con, null = ix.predicate("st_contains", poly, px, py)
    assert as_np(con).tolist() == [True, False, False, False, False, True, False]
    assert as_np(null).tolist() == [False] * 6 + [True]


@pytest.mark.parametrize("mode", ["auto", "direct"])
def test_st_covers_box_kats(gpu, mode):
    """SpatialRelationFunctionsTest.scala:113-139: st_covers(POLYGON((0 0,0 10,10 10,10 0,0 0)), p) is true
    for POINT(5 5), POINT(0 5) (edge) and POINT(0 0) (corner), false for POINT(-5 0) -- as the join
    condition and row by row."""
    from geomesa_amd.join import PolygonIndex, PolygonSet
    ps = PolygonSet.from_polygons([[[[(0, 0), (0, 10), (10, 10), (10, 0), (0, 0)]]]])
    ix = PolygonIndex(ps)
    px, py = [5.0, 0.0, 0.0, -5.0], [5.0, 5.0, 0.0, 0.0]
    pt, pl = ix.join(px, py, mode=mode, predicate="st_covers")
    assert sorted(as_np(pt).tolist()) == [0, 1, 2] and set(as_np(pl).tolist()) == {0}
    cov, null = ix.predicate("st_covers", [0, 0, 0, 0], px, py)
    assert as_np(cov).tolist() == [True, True, True, False]
    assert not as_np(null).any()
    pt, _ = ix.join(px, py, mode=mode, predicate="st_contains")   # :96-99, the same points under st_contains
    assert as_np(pt).tolist() == [0]


def _envelopes(ps):
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    env = []
    for p in range(ps.n_polys):
        a, b = rvo[pro[ppo[p]]], rvo[pro[ppo[p + 1]]]
        env.append((vx[a:b].min(), vy[a:b].min(), vx[a:b].max(), vy[a:b].max()))
    return np.array(env)


def oracle_pairs(oracle, ps, px, py, pred):
    ops = oracle.OraclePolySet(*ps.to_arrays())
    env = _envelopes(ps)
    out = set()
    for i, (x, y) in enumerate(zip(px, py)):
        cand = np.flatnonzero((env[:, 0] <= x) & (x <= env[:, 2]) & (env[:, 1] <= y) & (y <= env[:, 3]))
        for p in cand:
            if (ops.intersects if pred == "st_intersects" else ops.contains)(int(p), x, y):
                out.add((i, int(p)))
    return out


@pytest.mark.parametrize("mode", ["auto", "direct"])
@pytest.mark.parametrize("pred", ["st_intersects", "st_contains"])
def test_join_predicates_with_boundary_points(gpu, oracle, mode, pred):
    """The join condition's UDF (GeoMesaJoinRelation.scala:67-79): st_intersects keeps the points on
    polygon boundaries (vertices, edge midpoints) that st_contains drops."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(NX, NY)
    _, px, py = rows(ps, 30_000, seed=21)
    pt, pl = PolygonIndex(ps).join(px, py, mode=mode, predicate=pred)
    got = set(zip(as_np(pt).tolist(), as_np(pl).tolist()))
    exp = oracle_pairs(oracle, ps, px, py, pred)
    assert got == exp
    if pred == "st_intersects":
        assert len(exp) > len(oracle_pairs(oracle, ps, px, py, "st_contains")) + 500


def test_arrow_join_intersects(gpu, oracle):
    from geomesa_amd import arrow
    from geomesa_amd.join import synthetic_counties
    from test_gpu_arrow import point_array, polyset_to_arrow
    ps = synthetic_counties(NX, NY)
    _, px, py = rows(ps, 20_000, seed=5)
    ix = arrow.ArrowPolygonIndex(polyset_to_arrow(ps), kind="multipolygon")
    pt, pl = ix.join(point_array(px, py), predicate="st_intersects")
    assert set(zip(as_np(pt).tolist(), as_np(pl).tolist())) == oracle_pairs(oracle, ps, px, py, "st_intersects")


def test_relate_rows_deep_inside(gpu, oracle):
    """Rows deep inside their own county (points near each county's centre, where whole coarse cells are
    INTERIOR) and the same points against a neighbouring county, against the oracle."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(NX, NY)
    ix = PolygonIndex(ps)
    rng = np.random.default_rng(7)
    poly, px, py = [], [], []
    for p in range(ps.n_polys):
        r0 = ps.ring_vert_off[ps.part_ring_off[ps.poly_part_off[p]]]
        r1 = ps.ring_vert_off[ps.part_ring_off[ps.poly_part_off[p]] + 1]
        cx, cy = ps.vx[r0:r1].mean(), ps.vy[r0:r1].mean()
        px += list(cx + rng.uniform(-0.05, 0.05, 16)); py += list(cy + rng.uniform(-0.05, 0.05, 16)); poly += [p] * 16
    poly, px, py = np.array(poly, np.int32), np.array(px), np.array(py)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    exp = np.array([ops.locate(int(p), x, y) for p, x, y in zip(poly, px, py)], np.uint8)
    assert (exp == 2).mean() > 0.7   # (a tenth of the counties have a hole around the centre)
    assert np.array_equal(as_np(ix.relate(poly, px, py)), exp)
    other = ((poly + 1) % ps.n_polys).astype(np.int32)
    exp = np.array([ops.locate(int(p), x, y) for p, x, y in zip(other, px, py)], np.uint8)
    assert np.array_equal(as_np(ix.relate(other, px, py)), exp)


def test_relate_unaligned_and_odd_rows(gpu):
    """The row predicate reads two adjacent rows per lane when the columns are 16-B aligned and row by
    row otherwise: both layouts, and an odd row count (a last lane with one row), give the same locations."""
    import torch
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(NX, NY)
    poly, px, py = rows(ps, 40_001, seed=31)
    ix = PolygonIndex(ps)
    full = as_np(ix.relate(poly, px, py))
    dx = torch.as_tensor(px, device="cuda")
    dy = torch.as_tensor(py, device="cuda")
    shifted = as_np(ix.relate(poly[1:], dx[1:], dy[1:]))   # 8-B offset columns: the row-by-row loads
    assert np.array_equal(shifted, full[1:])
    odd = as_np(ix.relate(poly[:12_345], px[:12_345], py[:12_345]))
    assert np.array_equal(odd, full[:12_345])


@pytest.mark.parametrize("which", ["lattice", "stacked"])
@pytest.mark.parametrize("cells,host", [(0, False), (64, False), (16384, False), (0, True)])
def test_relate_and_join_lattice_exact(gpu, cells, host, which):
    """The kernels against exact rational arithmetic (tests/test_oracle_exact.py): lattice polygons
    with holes and MultiPolygon parts sharing an edge / a vertex, every lattice point on multiples of
    1/8 -- thousands exactly on edges and vertices.  Row predicate: the location per row; join: the
    st_contains pairs."""
    from geomesa_amd.join import PolygonIndex, PolygonSet
    from test_oracle_exact import exact_lattice
    polys, px, py, exp = exact_lattice(which)
    ps = PolygonSet.from_polygons(polys)
    from geomesa_amd import _lib
    ctx = _lib.context()
    try:   # the device build (default) and the host build (GM_PARAM_INDEX_BUILD = 1)
        ctx.set_param(_lib.GM_PARAM_INDEX_BUILD, 1 if host else 0)
        ix = PolygonIndex(ps, ctx, cells)
    finally:
        ctx.set_param(_lib.GM_PARAM_INDEX_BUILD, 0)
    n = len(px)
    poly = np.repeat(np.arange(len(polys), dtype=np.int32), n)
    for wide in (False, True):
        with rows64(wide):
            loc = as_np(ix.relate(poly, np.tile(px, len(polys)), np.tile(py, len(polys))))
        assert np.array_equal(loc, exp.ravel()), (wide, np.flatnonzero(loc != exp.ravel())[:10])
    pt, pl = ix.join(px, py)
    got = set(zip(as_np(pt).tolist(), as_np(pl).tolist()))
    want = {(i, p) for p in range(len(polys)) for i in np.flatnonzero(exp[p] == 2).tolist()}
    assert got == want
    pt, pl = ix.join(px, py, predicate="st_intersects")
    got = set(zip(as_np(pt).tolist(), as_np(pl).tolist()))
    want = {(i, p) for p in range(len(polys)) for i in np.flatnonzero(exp[p] != 0).tolist()}
    assert got == want
    assert (exp == 1).sum() > 300


def test_relate_us_states_shared_borders(gpu, oracle):
    """Real polygons whose neighbours share borders (the reference's us_state shapefile fixture): cells
    on a border list two or more polygons with BOUNDARY entries, the case the list search
    (list_poly) decides.  Rows: random points with the state of a neighbouring point, plus every
    vertex with its own state and with a random other state."""
    from geomesa_amd.join import PolygonIndex
    from shapefile import us_states
    ps, _ = us_states()
    rng = np.random.default_rng(29)
    n = 200_000
    px = rng.uniform(-125.0, -66.0, n); py = rng.uniform(24.0, 50.0, n)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    pt, pl = ops.join(px, py, nthreads=8, predicate="st_intersects")
    poly = rng.integers(0, ps.n_polys, n).astype(np.int32)
    poly[pt] = pl                                      # the point's own state where it has one
    shift = np.roll(np.arange(n), 1)
    poly[::3] = poly[shift[::3]]                       # a neighbouring point's state (often a border pair)
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    vi = rng.choice(len(vx), 10_000, replace=False)
    vpoly = np.searchsorted(np.asarray(ppo)[1:], np.searchsorted(np.asarray(pro)[1:], np.searchsorted(np.asarray(rvo)[1:], vi, side="right"), side="right"), side="right").astype(np.int32)
    vpoly[1::2] = rng.integers(0, ps.n_polys, len(vpoly[1::2]))
    poly = np.concatenate([poly, vpoly]); px = np.concatenate([px, vx[vi]]); py = np.concatenate([py, vy[vi]])
    for cells, wide in ((0, False), (4096, False), (4096, True)):
        with rows64(wide):
            loc = as_np(PolygonIndex(ps, cells_per_poly=cells).relate(poly, px, py))
        exp = np.array([ops.locate(int(p), x, y) for p, x, y in zip(poly, px, py)], np.uint8)
        assert np.array_equal(loc, exp), (cells, np.flatnonzero(loc != exp)[:10])
        assert (exp == 1).sum() > 4_000 and (exp == 2).sum() > 50_000
