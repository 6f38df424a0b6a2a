"""The join on real polygons: the reference's US-state shapefile fixture (52 records, 132 rings,
13,832 vertices; geomesa-convert-shp/src/test/resources/us_state/cb_2017_us_state_20m.shp, read by
tests/shapefile.py), against the oracle for both join predicates (SpatialRelationFunctions.scala:29
st_contains, :34 st_intersects), plus join passes forced across chunk boundaries (GM_PARAM_JOIN_CHUNK,
even and odd chunk sizes)."""
import numpy as np
import pytest

from shapefile import us_states
from test_gpu_scan_join_ranges import _sorted_pairs, as_np

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module")
def states():
    ps, rows = us_states()
    return ps, rows


def state_points(ps, n=2_000_000, seed=21):
    """n uniform CONUS-box points, every state vertex, every edge midpoint, and points a hair off
    the vertices (near-collinear orientation cases)."""
    rng = np.random.default_rng(seed)
    px = rng.uniform(-125.0, -66.0, n)
    py = rng.uniform(24.0, 50.0, n)
    mx, my = (ps.vx[1:] + ps.vx[:-1]) / 2, (ps.vy[1:] + ps.vy[:-1]) / 2
    jx, jy = np.nextafter(ps.vx, np.inf), np.nextafter(ps.vy, -np.inf)
    return np.concatenate([px, ps.vx, mx, jx]), np.concatenate([py, ps.vy, my, jy])


def test_states_fixture_shape(states):
    ps, rows = states
    assert ps.n_polys == 52 and len(ps.ring_vert_off) - 1 == 132 and ps.n_vertices == 13_832
    assert sorted(r["STUSPS"] for r in rows)[:3] == ["AK", "AL", "AR"]


@pytest.mark.parametrize("predicate", ["st_contains", "st_intersects"])
def test_states_join_parity(gpu, oracle, states, predicate):
    from geomesa_amd.join import PolygonIndex
    ps, _ = states
    px, py = state_points(ps)
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=16, predicate=predicate)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    ix = PolygonIndex(ps)
    pt, pl = ix.join(px, py, predicate=predicate)
    assert np.array_equal(_sorted_pairs(pt, pl), exp), predicate
    # a vertex point lies on its own state's boundary: never contained by it; on shared borders it
    # intersects two states
    n0 = len(px) - (3 * ps.n_vertices - 1)   # first vertex point (after n random points)
    on_vertex = (exp[:, 0] >= n0) & (exp[:, 0] < n0 + ps.n_vertices)
    if predicate == "st_contains":
        ring_of = np.repeat(np.arange(len(ps.ring_vert_off) - 1), np.diff(ps.ring_vert_off))
        part_of = np.repeat(np.arange(len(ps.part_ring_off) - 1), np.diff(ps.part_ring_off))
        poly_of = np.repeat(np.arange(ps.n_polys), np.diff(ps.poly_part_off))
        owner = poly_of[part_of[ring_of]]
        v = exp[on_vertex]
        assert not (owner[v[:, 0] - n0] == v[:, 1]).any()
    else:
        ids, cnt = np.unique(exp[on_vertex, 0], return_counts=True)
        assert len(ids) == ps.n_vertices and (cnt >= 2).sum() > 100


def test_states_city_kats_gpu(gpu, states):
    """Known answers independent of both implementations: inland points of named places."""
    from geomesa_amd.join import PolygonIndex
    ps, rows = states
    pts = {"CO": (-104.99, 39.74), "TX": (-97.74, 30.27), "HI": (-157.98, 21.45), "AK": (-147.72, 64.84),
           "PR": (-66.5, 18.2), "IL": (-89.65, 39.78), "DC": (-77.03, 38.90), "ME": (-69.0, 45.5)}
    names = list(pts)
    pt, pl = PolygonIndex(ps).join([pts[k][0] for k in names], [pts[k][1] for k in names])
    got = {names[i]: rows[p]["STUSPS"] for i, p in zip(as_np(pt).tolist(), as_np(pl).tolist())}
    assert got == {k: k for k in names}


@pytest.mark.parametrize("chunk", [400_000, 399_999, 131_071])
@pytest.mark.parametrize("fixture", ["states", "counties"])
def test_join_across_chunks(gpu, oracle, states, chunk, fixture):
    """GM_PARAM_JOIN_CHUNK forces >= 3 passes: per-pass id offsets, pair counters carried across
    passes, and the capacity path.  Odd chunk sizes are rounded down to even, so every chunk of the
    16-B aligned columns keeps the 16-B pair loads aligned."""
    from geomesa_amd import _lib
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    if fixture == "states":
        ps = states[0]
        px, py = state_points(ps, n=1_500_000, seed=5)
    else:
        ps = synthetic_counties(20, 10)
        px, py = synthetic_points(1_500_000, seed=6)
    n = len(px)
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=16)
    exp = np.stack([opt + 77, opl.astype(np.int64)], 1)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    ix = PolygonIndex(ps)
    ctx = ix.ctx
    assert (n + chunk - 1) // chunk >= 3
    try:
        ctx.set_param(_lib.GM_PARAM_JOIN_CHUNK, chunk)
        assert ctx.get_param(_lib.GM_PARAM_JOIN_CHUNK) == chunk
        pt, pl = ix.join(px, py, id_base=77)
        assert np.array_equal(_sorted_pairs(pt, pl), exp)
        assert ix.join(px, py, id_base=77, count_only=True) == len(exp)
        pt2, _ = ix.join(px, py, id_base=77, cap=100)   # GM_E_CAPACITY, then the retry
        assert len(pt2) == len(exp)
        # an unaligned column view (scalar loads) across the same chunks
        pt3, pl3 = ix.join(px[1:], py[1:], id_base=78)
        assert np.array_equal(_sorted_pairs(pt3, pl3), exp[exp[:, 0] >= 78])
    finally:
        ctx.set_param(_lib.GM_PARAM_JOIN_CHUNK, 0)
