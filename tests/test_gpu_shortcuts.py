"""GPU parity at the boundary shortcuts' decision thresholds (gm_pip.hip "Boundary shortcuts"): the
join and the row-wise predicate locate a point of a cell crossed by one or two segments from the
segments' quantized lines when it is at least SC_T (6 / 16384 of a cell) from every line, and from the
blob otherwise.  Points are put on both sides of every edge (perpendicular offsets from the edge's
midpoint) and around every vertex, at distances from 1e-12 deg to 1e-2 deg -- across the threshold
at every grid density used here -- and compared with the oracle (JTS PointLocator restatement,
geomesa-spark-jts/.../udf/SpatialRelationFunctions.scala:29 semantics; parity unpinned beyond the
reference's box KATs)."""
import numpy as np
import pytest

from test_gpu_scan_join_ranges import _sorted_pairs, as_np

pytestmark = pytest.mark.gpu

OFFSETS = np.array([1e-12, 1e-10, 1e-8, 1e-7, 1e-6, 3e-6, 1e-5, 2e-5, 5e-5, 1e-4, 3e-4, 1e-3, 1e-2])


def threshold_points(ps, stride=1):
    """Per edge (every stride-th): the midpoint moved +-d along the edge normal; per vertex: the
    vertex moved +-d along both axes and both diagonals; d over OFFSETS."""
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    xs, ys = [], []
    for r in range(len(rvo) - 1):
        a, b = rvo[r], rvo[r + 1]
        x, y = vx[a:b], vy[a:b]
        ex, ey = x[1:] - x[:-1], y[1:] - y[:-1]
        ln = np.hypot(ex, ey)
        ok = ln > 0
        nx, ny = -ey[ok] / ln[ok], ex[ok] / ln[ok]
        mx, my = (0.5 * (x[1:] + x[:-1]))[ok], (0.5 * (y[1:] + y[:-1]))[ok]
        mx, my, nx, ny = mx[::stride], my[::stride], nx[::stride], ny[::stride]
        for d in OFFSETS:
            for s in (1.0, -1.0):
                xs.append(mx + s * d * nx); ys.append(my + s * d * ny)
        px, py = x[:-1][::stride], y[:-1][::stride]
        for d in OFFSETS[::2]:
            for ux, uy in ((1, 0), (-1, 0), (0, 1), (0, -1), (0.7071, 0.7071), (-0.7071, 0.7071)):
                xs.append(px + d * ux); ys.append(py + d * uy)
    return np.concatenate(xs), np.concatenate(ys)


@pytest.mark.parametrize("grid,cells", [((20, 10), 0), ((20, 10), 2048), ((80, 40), 0)])
@pytest.mark.parametrize("predicate", ["st_contains", "st_intersects"])
def test_join_at_shortcut_thresholds(gpu, oracle, grid, cells, predicate):
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(*grid)
    px, py = threshold_points(ps, stride=1 if grid[0] <= 20 else 7)
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=16, predicate=predicate)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    ix = PolygonIndex(ps, cells_per_poly=cells)
    pt, pl = ix.join(px, py, predicate=predicate)
    assert np.array_equal(_sorted_pairs(pt, pl), exp), len(exp)


def test_relate_at_shortcut_thresholds(gpu, oracle):
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(12, 6)
    px, py = threshold_points(ps, stride=3)
    px, py = np.concatenate([px, ps.vx[::5]]), np.concatenate([py, ps.vy[::5]])   # + vertices: boundary rows
    ops = oracle.OraclePolySet(*ps.to_arrays())
    # the polygon that owns each point's edge or vertex: nearest polygon centroid works for this layout
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    ring_of = np.repeat(np.arange(len(rvo) - 1), np.diff(rvo))
    part_of = np.repeat(np.arange(len(pro) - 1), np.diff(pro))
    poly_of = np.repeat(np.arange(ps.n_polys), np.diff(ppo))[part_of[ring_of]]
    cx = np.bincount(poly_of, vx) / np.bincount(poly_of)
    cy = np.bincount(poly_of, vy) / np.bincount(poly_of)
    near = np.argmin((px[:, None] - cx[None, :]) ** 2 + (py[:, None] - cy[None, :]) ** 2, 1).astype(np.int32)
    loc = as_np(PolygonIndex(ps).relate(near, px, py))
    exp = np.array([ops.locate(int(p), x, y) for p, x, y in zip(near, px, py)], np.uint8)
    assert np.array_equal(loc, exp)
    assert (exp == 1).sum() > 0 and (exp == 2).sum() > 0 and (exp == 0).sum() > 0


@pytest.mark.parametrize("fmt", [0, 1])
def test_join_coarse_mask_formats(gpu, oracle, fmt):
    """Both layouts of the join's coarse sub-block masks (gm_pip.hpp coarse_mask): EMPTY bits of 16
    sub-blocks (any polygon count) and EMPTY / INTERIOR(main) bits of 8 (fewer than 2^14 polygons),
    forced through GM_PARAM_INDEX_COARSE at index build, against the oracle on random and boundary
    points, for the join and the row predicate."""
    from geomesa_amd import _lib
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(20, 10)
    px, py = synthetic_points(300_000, seed=9)
    tx, ty = threshold_points(ps, stride=5)
    px, py = np.concatenate([px, tx]), np.concatenate([py, ty])
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=16)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    ctx = _lib.context()
    try:
        ctx.set_param(_lib.GM_PARAM_INDEX_COARSE, fmt)
        ix = PolygonIndex(ps)
    finally:
        ctx.set_param(_lib.GM_PARAM_INDEX_COARSE, -1)
    pt, pl = ix.join(px, py)
    assert np.array_equal(_sorted_pairs(pt, pl), exp), fmt
    # the row predicate over the same index: each point against the polygon the oracle pairs it with
    # (INTERIOR) and against polygon 0 (mostly EXTERIOR)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    rows = np.concatenate([exp[:2000, 1], np.zeros(2000, np.int64)]).astype(np.int32)
    rx = np.concatenate([px[exp[:2000, 0]], px[:2000]]); ry = np.concatenate([py[exp[:2000, 0]], py[:2000]])
    loc = as_np(ix.relate(rows, rx, ry))
    assert np.array_equal(loc, np.array([ops.locate(int(p), x, y) for p, x, y in zip(rows, rx, ry)], np.uint8))


def test_join_census_accounts_for_every_point(gpu):
    """gm_pip_join_census (diagnostic): every point ends at exactly one stage of the lookup chain."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(20, 10)
    px, py = synthetic_points(300_000)
    px = np.concatenate([px, [np.nan, 0.0, -200.0]]); py = np.concatenate([py, [30.0, np.nan, 30.0]])
    c = PolygonIndex(ps).census(px, py)
    assert c["points"] == len(px)
    assert c["points"] == c["outside"] + c["coarse_empty"] + c["coarse_interior"] + c["fine"]
    assert c["fine"] == (c["fine_empty"] + c["fine_interior"] + c["fine_line"] + c["fine_compact"] + c["fine_generic"]
                         + c["fine_list"] + c["fine_inline"])
    assert c["fine_inline"] > c["fine_inline2"] > 0 and c["inline_fallback"] < c["fine_inline"]
    assert c["coarse_gather"] <= c["points"] - c["outside"]
    assert c["fine_line"] == c["line_resolved"] + c["line_fallback"]
    assert c["outside"] >= 3 and c["fine"] > 0 and c["coarse_interior"] > 0
