"""GPU parity for Arrow columnar input: keys and the join read geomesa-arrow-jts
vectors in place, bit-exact against the oracle's per-row restatement (oracle.arrow_*) and against the
column entry points on the de-interleaved coordinates."""
import numpy as np
import pyarrow as pa
import pytest

from test_gpu_parity import T2020, T2021, as_np, edge_points

pytestmark = pytest.mark.gpu

PT = pa.list_(pa.float64(), 2)
PT4 = pa.list_(pa.float32(), 2)


def point_array(x, y, null_mask=None, f32=False, flip=False):
    a, b = (x, y) if flip else (y, x)
    flat = np.stack([a, b], 1).reshape(-1).astype(np.float32 if f32 else np.float64)
    mask = None if null_mask is None else pa.array(null_mask)
    return pa.FixedSizeListArray.from_arrays(pa.array(flat), 2, mask=mask)


def time_array(t, null_mask=None):
    return pa.array(t, pa.timestamp("ms"), mask=null_mask)


def expect_z3(oracle, x, y, t, nulls, tnulls, lenient, period):
    tt = np.where(tnulls, 0, t) if tnulls is not None else t
    b, z, st = oracle.z3_index_key_batch(x, y, tt, lenient, period)
    if nulls is not None:
        b = np.where(nulls, 0, b); z = np.where(nulls, 0, z); st = np.where(nulls, oracle.NULL_GEOM, st)
    return b, z, st


@pytest.mark.parametrize("period", [0, 1, 2, 3])
@pytest.mark.parametrize("lenient", [False, True])
def test_z3_keys_arrow_edges(gpu, oracle, period, lenient):
    from geomesa_amd import arrow
    x, y, t = edge_points()
    n = len(x)
    rng = np.random.default_rng(5)
    nulls = rng.uniform(size=n) < 0.1
    tnulls = rng.uniform(size=n) < 0.1
    b, z, st = arrow.z3_index_keys(point_array(x, y, nulls), time_array(t, tnulls), period=period,
                                   lenient=lenient, status=True)
    ob, oz, ost = expect_z3(oracle, x, y, t, nulls, tnulls, lenient, period)
    assert np.array_equal(as_np(st), ost)
    assert np.array_equal(as_np(b), ob) and np.array_equal(as_np(z), oz)


@pytest.mark.parametrize("f32", [False, True])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("n", [0, 1, 7, 100_001])
def test_z3_keys_arrow_random(gpu, oracle, f32, flip, n):
    from geomesa_amd import arrow
    rng = np.random.default_rng(n + 11)
    x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n); t = rng.integers(T2020, T2021, n)
    if f32:   # the Float4 vectors widen their floats (readOrdinal)
        x = x.astype(np.float32).astype(np.float64); y = y.astype(np.float32).astype(np.float64)
    nulls = rng.uniform(size=n) < 0.05
    b, z, st = arrow.z3_index_keys(point_array(x, y, nulls, f32, flip), time_array(t), status=True,
                                   flip_axis=flip)
    ob, oz, ost = expect_z3(oracle, x, y, t, nulls, None, False, 1)
    assert np.array_equal(as_np(st), ost)
    assert np.array_equal(as_np(b), ob) and np.array_equal(as_np(z), oz)


def test_z3_keys_arrow_slices_and_null_dtg_column(gpu, oracle):
    from geomesa_amd import arrow
    rng = np.random.default_rng(2)
    n = 5000
    x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n); t = rng.integers(T2020, T2021, n)
    nulls = rng.uniform(size=n) < 0.1
    pts, ts = point_array(x, y, nulls), time_array(t)
    for a, m in [(1, 4001), (3, 2), (17, 0), (999, 4000)]:   # unaligned starts: scalar paths
        b, z, st = arrow.z3_index_keys(pts.slice(a, m), ts.slice(a, m), status=True)
        ob, oz, ost = expect_z3(oracle, x[a:a + m], y[a:a + m], t[a:a + m], nulls[a:a + m], None, False, 1)
        assert np.array_equal(as_np(st), ost) and np.array_equal(as_np(z), oz) and np.array_equal(as_np(b), ob)
    b, z, st = arrow.z3_index_keys(pts, None, status=True)   # no date attribute value: time 0
    ob, oz, ost = expect_z3(oracle, x, y, np.zeros(n, np.int64), nulls, None, False, 1)
    assert np.array_equal(as_np(z), oz) and np.array_equal(as_np(b), ob)


def test_z3_keys_arrow_matches_row_oracle_and_raises(gpu, oracle):
    from geomesa_amd import arrow
    from geomesa_amd.curve import IllegalArgumentException
    vals = [[10.0, 20.0], None, [-91.0, 0.0], [45.5, -120.25]]
    pts = pa.array(vals, PT)
    ts = pa.array([T2020, None, T2020, -5], pa.timestamp("ms"))
    b, z, st = arrow.z3_index_keys(pts, ts, status=True)
    ob, oz, ost = oracle.arrow_z3_keys(pts, ts)
    assert as_np(st).tolist() == ost.tolist() == [0, 4, 1, 2]
    assert np.array_equal(as_np(z), oz) and np.array_equal(as_np(b), ob)
    with pytest.raises(IllegalArgumentException, match="Null geometry"):
        arrow.z3_index_keys(pts.slice(0, 2), ts.slice(0, 2))
    bb, zz = arrow.z3_index_keys(pts.slice(0, 1), ts.slice(0, 1))
    assert as_np(zz)[0] == oz[0]


@pytest.mark.parametrize("lenient", [False, True])
def test_z2_keys_arrow(gpu, oracle, lenient):
    from geomesa_amd import arrow
    x, y, _ = edge_points()
    x, y = x[::16], y[::16]
    rng = np.random.default_rng(9)
    x = np.concatenate([x, rng.uniform(-180, 180, 30001)]); y = np.concatenate([y, rng.uniform(-90, 90, 30001)])
    nulls = rng.uniform(size=len(x)) < 0.05
    z, st = arrow.z2_index_keys(point_array(x, y, nulls), lenient=lenient, status=True)
    oz, ost = oracle.z2_index_batch(x, y, lenient)
    oz = np.where(nulls, 0, oz); ost = np.where(nulls, oracle.NULL_GEOM, ost)
    assert np.array_equal(as_np(st), ost) and np.array_equal(as_np(z), oz)


def test_points_to_columns(gpu):
    from geomesa_amd import arrow
    rng = np.random.default_rng(4)
    n = 10001
    x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n)
    nulls = rng.uniform(size=n) < 0.1
    gx, gy = arrow.points_to_columns(point_array(x, y, nulls))
    assert np.array_equal(as_np(gx), np.where(nulls, np.nan, x), equal_nan=True)
    assert np.array_equal(as_np(gy), np.where(nulls, np.nan, y), equal_nan=True)


# ------------------------------------------------------------------ envelopes -> XZ keys

TYPES = {
    "linestring": pa.list_(PT), "multipoint": pa.list_(PT), "polygon": pa.list_(pa.list_(PT)),
    "multilinestring": pa.list_(pa.list_(PT)), "multipolygon": pa.list_(pa.list_(pa.list_(PT))),
}
DEPTH = {"linestring": 1, "multipoint": 1, "polygon": 2, "multilinestring": 2, "multipolygon": 3}


def rand_geoms(rng, kind, n, null_frac=0.05):
    def tup():
        # log-uniform extents around a world-uniform centre, some outside the world (lenient cases)
        return [float(rng.uniform(-95, 95)), float(rng.uniform(-185, 185))]

    def local(c, s):
        return [c[0] + float(rng.uniform(-s, s)), c[1] + float(rng.uniform(-s, s))]

    def geom(depth, c, s):
        if depth == 0:
            return local(c, s)
        k = int(rng.integers(0 if depth == DEPTH[kind] else 1, 5))
        return [geom(depth - 1, c, s) for _ in range(k)]
    out = []
    for _ in range(n):
        if rng.uniform() < null_frac:
            out.append(None)
            continue
        out.append(geom(DEPTH[kind], tup(), 10 ** rng.uniform(-6, 1)))
    return pa.array(out, TYPES[kind])


@pytest.mark.parametrize("kind", sorted(TYPES))
@pytest.mark.parametrize("lenient", [False, True])
def test_xz2_keys_arrow(gpu, oracle, kind, lenient):
    from geomesa_amd import arrow
    rng = np.random.default_rng(len(kind) * 31 + lenient)
    arr = rand_geoms(rng, kind, 3000).slice(5)
    xz, st = arrow.xz2_index_keys(arr, kind=kind, lenient=lenient, status=True)
    oz, ost = oracle.arrow_xz2_keys(arr, kind, lenient=lenient)
    assert np.array_equal(as_np(st), ost)
    assert np.array_equal(as_np(xz), oz)


@pytest.mark.parametrize("kind", ["linestring", "polygon", "multipolygon"])
@pytest.mark.parametrize("period", [0, 1, 3])
def test_xz3_keys_arrow(gpu, oracle, kind, period):
    from geomesa_amd import arrow
    rng = np.random.default_rng(period * 7 + len(kind))
    arr = rand_geoms(rng, kind, 2000)
    t = rng.integers(T2020, T2021, len(arr))
    t[::97] = -1                       # BinnedTime throws even when lenient
    ts = pa.array(t, pa.timestamp("ms"), mask=rng.uniform(size=len(arr)) < 0.05)
    b, xz, st = arrow.xz3_index_keys(arr, ts, kind=kind, period=period, lenient=True, status=True)
    ob, oz, ost = oracle.arrow_xz3_keys(arr, ts, kind, period=period, lenient=True)
    assert np.array_equal(as_np(st), ost)
    assert np.array_equal(as_np(xz), oz) and np.array_equal(as_np(b), ob)


def test_xz_keys_arrow_match_envelope_columns(gpu, oracle):
    """A polygon column's keys equal gm_xz2_index over the envelopes the oracle computes."""
    from geomesa_amd import arrow
    from geomesa_amd.curve import XZ2SFC
    rng = np.random.default_rng(12)
    arr = rand_geoms(rng, "polygon", 20000, null_frac=0.0)
    rows = oracle.arrow_rows(arr, "polygon")
    env = np.array([oracle.jts_envelope(r, "polygon") for r in rows])
    ok = env[:, 0] <= env[:, 2]
    xz, st = arrow.xz2_index_keys(arr, kind="polygon", lenient=True, status=True)
    ref = XZ2SFC(12).index(env[ok, 0], env[ok, 1], env[ok, 2], env[ok, 3], lenient=True)
    assert np.array_equal(as_np(xz)[ok], as_np(ref))


# ------------------------------------------------------------------ join over Arrow columns

def polyset_to_arrow(ps, f32=False):
    """A PolygonSet as a geomesa-arrow-jts MultiPolygon column ([y, x] tuples)."""
    vals = []
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    for p in range(ps.n_polys):
        parts = []
        for q in range(ppo[p], ppo[p + 1]):
            parts.append([[[float(vy[j]), float(vx[j])] for j in range(rvo[r], rvo[r + 1])]
                          for r in range(pro[q], pro[q + 1])])
        vals.append(parts)
    return pa.array(vals, pa.list_(pa.list_(pa.list_(PT4 if f32 else PT))))


@pytest.mark.parametrize("mode", ["auto", "direct"])
def test_join_arrow_matches_columns(gpu, oracle, mode):
    from geomesa_amd import arrow
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(12, 6)
    px, py = synthetic_points(200_001)
    rng = np.random.default_rng(1)
    nulls = rng.uniform(size=len(px)) < 0.05
    idx = arrow.ArrowPolygonIndex(polyset_to_arrow(ps), kind="multipolygon")
    pt, pl = idx.join(point_array(px, py, nulls), mode=mode)
    got = set(zip(as_np(pt).tolist(), as_np(pl).tolist()))
    ept, epl = PolygonIndex(ps).join(px, py)
    exp = {(a, b) for a, b in zip(as_np(ept).tolist(), as_np(epl).tolist()) if not nulls[a]}
    assert got == exp
    assert idx.join(point_array(px, py, nulls), count_only=True, mode=mode) == len(exp)


def test_join_arrow_against_oracle_with_null_polygon(gpu, oracle):
    from geomesa_amd import arrow
    from geomesa_amd.join import synthetic_counties, synthetic_points
    ps = synthetic_counties(6, 3)
    arr = polyset_to_arrow(ps)
    # null out polygon 4: it never matches
    mask = np.zeros(ps.n_polys, bool); mask[4] = True
    arr = pa.ListArray.from_arrays(arr.offsets, arr.values, mask=pa.array(mask))
    px, py = synthetic_points(30_000)
    pt, pl = arrow.ArrowPolygonIndex(arr, kind="multipolygon").join(point_array(px, py))
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py)
    exp = {(a, b) for a, b in zip(opt.tolist(), opl.tolist()) if b != 4}
    assert set(zip(as_np(pt).tolist(), as_np(pl).tolist())) == exp
