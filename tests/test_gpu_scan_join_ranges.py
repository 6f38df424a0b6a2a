"""GPU parity for the filter scans, the st_contains join and batched range decomposition."""
import numpy as np
import pytest

from test_host_planning import IDX_STRATEGY_KATS, idx_strategy_features, ms
from geomesa_amd import filters as F
from geomesa_amd.keyspace import Z3IndexKeySpace, during

pytestmark = pytest.mark.gpu

T2020, T2021 = 1577836800000, 1609459200000


def as_np(t):
    return t.detach().cpu().numpy()


# ---------------------------------------------------------------- Z3Filter scan
@pytest.mark.parametrize("bbox,interval,expected", IDX_STRATEGY_KATS)
def test_idx_strategy_kats_gpu(gpu, bbox, interval, expected):  # Z3IdxStrategyTest.scala:96-181
    feats = idx_strategy_features()
    ids = np.array([f[0] for f in feats])
    ks = Z3IndexKeySpace()
    b, z = ks.sfc.index_keys([f[1] for f in feats], [f[2] for f in feats], [f[3] for f in feats])
    v = ks.get_index_values([bbox], [interval])
    m, got, n = F.scan(F.Z3Filter.from_values(v), b, z, ks.bin_ranges(v), want_ids=True)
    assert set(ids[as_np(got)].tolist()) == expected and n == len(expected)


def random_keys(n, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n); t = rng.integers(T2020, T2021, n)
    return x, y, t


QUERIES = [
    ([(-10, 35, 30, 60)], during(ms("2020-06-01T00:00:00.000Z"), ms("2020-06-08T12:00:00.000Z"))),
    ([(-10, 35, 30, 60), (100, -40, 120, -10)], during(ms("2020-03-01T00:00:00.000Z"), ms("2020-05-08T12:00:00.000Z"))),
    ([(-180, -90, 180, 90)], during(ms("2020-12-30T00:00:00.000Z"), ms("2021-01-01T00:00:00.000Z"))),
    ([(0.0, 0.0, 0.5, 0.5)], during(ms("2020-01-01T00:00:00.000Z"), ms("2020-01-01T00:00:00.500Z"))),
]


@pytest.mark.parametrize("q", QUERIES)
def test_z3filter_scan_parity(gpu, oracle, q):
    import torch
    x, y, t = random_keys(1_000_003)
    ks = Z3IndexKeySpace()
    b, z = ks.sfc.index_keys(x, y, t)
    v = ks.get_index_values(q[0], [q[1]])
    f = F.Z3Filter.from_values(v)
    br = ks.bin_ranges(v)
    m, ids, n = F.scan(f, b, z, br, want_ids=True)
    om = oracle.z3filter_scan(F.serialize_to_bytes(f), br, as_np(b), as_np(z))
    assert np.array_equal(as_np(m), om)
    assert np.array_equal(as_np(ids), np.nonzero(om)[0]) and n == int(om.sum())
    # no bin restriction (UnboundedRange) and count only
    m2, _, n2 = F.scan(f, b, z, [])
    om2 = oracle.z3filter_scan(F.serialize_to_bytes(f), [], as_np(b), as_np(z))
    assert np.array_equal(as_np(m2), om2) and n2 == int(om2.sum())
    # ids capacity smaller than the match count: GM_E_CAPACITY path keeps the first ids
    if n > 4:
        _, ids3, n3 = F.scan(f, b, z, br, want_ids=True, ids_cap=3)
        assert n3 == n and np.array_equal(as_np(ids3), np.nonzero(om)[0][:3])
    del torch


def test_z2filter_scan_parity(gpu, oracle):
    from geomesa_amd.curve import Z2SFC
    from geomesa_amd.keyspace import Z2IndexKeySpace
    x, y, _ = random_keys(500_001, seed=4)
    z = Z2SFC().index(x, y)
    f = F.Z2Filter.from_values(Z2IndexKeySpace().get_index_values([(-10, 35, 30, 60), (5, 5, 6, 6)]))
    m, ids, n = F.z2_scan(f, z, want_ids=True)
    om = oracle.z2filter_scan(F.z2_serialize_to_bytes(f), as_np(z))
    assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])


@pytest.mark.parametrize("with_during", [False, True])
def test_strict_scan_parity(gpu, oracle, with_during):
    x, y, t = random_keys(777_777, seed=6)
    x[:5] = [-10, 30, -10, 30.0000001, 0]; y[:5] = [35, 60, 60, 35, 34.9999999]    # edges: inclusive BBOX
    t[:3] = [ms("2020-06-01T00:00:00.000Z"), ms("2020-06-08T12:00:00.000Z"), ms("2020-06-01T00:00:00.001Z")]
    bbox = (-10, 35, 30, 60)
    dur = (ms("2020-06-01T00:00:00.000Z"), ms("2020-06-08T12:00:00.000Z")) if with_during else None
    m, ids, n = F.strict_scan(x, y, t, bbox, dur, want_ids=True)
    om = oracle.strict_scan(x, y, t, bbox, dur)
    assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])


@pytest.mark.parametrize("n", [1, 7, 8, 63, 64, 65, 2047, 2048, 2049, 100_003])
def test_scans_ragged_and_unaligned(gpu, oracle, n):
    """Vectorised scans (8 rows per lane, 16-B loads) at ragged sizes, and the scalar kernels they
    fall back to when a column is not 16-B aligned (a view starting one row in)."""
    import torch
    x, y, t = random_keys(n + 1, seed=n)
    ks = Z3IndexKeySpace()
    q = QUERIES[1]
    v = ks.get_index_values(q[0], [q[1]])
    f = F.Z3Filter.from_values(v)
    fb = F.serialize_to_bytes(f)
    br = ks.bin_ranges(v)
    b, z = ks.sfc.index_keys(x, y, t)
    from geomesa_amd.curve import Z2SFC
    from geomesa_amd.keyspace import Z2IndexKeySpace
    z2 = Z2SFC().index(x, y)
    f2 = F.Z2Filter.from_values(Z2IndexKeySpace().get_index_values([(-10, 35, 30, 60), (100, -40, 120, -10)]))
    dx, dy, dt = (torch.from_numpy(a).cuda() for a in (x, y, t))
    bbox, dur = (-10, 35, 30, 60), (ms("2020-03-01T00:00:00.000Z"), ms("2020-05-08T12:00:00.000Z"))
    for off in (0, 1):   # off = 1: misaligned views -> scalar kernels
        sl = slice(off, off + n)
        m, ids, k = F.scan(f, b[sl], z[sl], br, want_ids=True)
        om = oracle.z3filter_scan(fb, br, as_np(b)[sl], as_np(z)[sl])
        assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0]) and k == int(om.sum())
        m, ids, k = F.z2_scan(f2, z2[sl], want_ids=True)
        om = oracle.z2filter_scan(F.z2_serialize_to_bytes(f2), as_np(z2)[sl])
        assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0]) and k == int(om.sum())
        for d in (None, dur):
            m, ids, k = F.strict_scan(dx[sl], dy[sl], dt[sl], bbox, d, want_ids=True)
            om = oracle.strict_scan(x[sl], y[sl], t[sl], bbox, d)
            assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])


ADVERSARIAL_Z3 = [
    # boxes past the 21-bit range, negative, empty (min > max), whole-range; epochs with null, empty
    # and multi-interval entries (Z3Filter.scala:31-62 decodes any row bytes, valid key or not)
    F.Z3Filter([[-5, 100, 3_000_000, 2_000_000], [10, 10, 5, 5], [0, 0, 2097151, 2097151]],
               [[[0, 1000], [500_000, 2_097_151]], None, [], [[-3, 7]]], 3, 6),
    F.Z3Filter([[2_000_000, -1, 2_097_152, 10]], [[[5, 5]]], -1, -1),
    F.Z3Filter([[0, 0, 0, 0], [7, 7, 7, 7]], [], 32767, -32768),
]


@pytest.mark.parametrize("k", range(len(ADVERSARIAL_Z3)))
def test_filters_on_arbitrary_row_bits(gpu, oracle, k):
    """Dilated-bound fast paths vs the oracle on arbitrary 64-bit z words (sign bit, bit 62 and 63
    set) and int16 bins, with filter bounds outside the dimension ranges."""
    rng = np.random.default_rng(31 + k)
    n = 300_001
    z = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    z[:4096] &= 0x7FFFFFFF  # small coordinates: boxes near 0 hit
    b = rng.integers(-4, 10, n).astype(np.int16)
    f = ADVERSARIAL_Z3[k]
    for br in ([], [(2, 4)], [(-4, -1), (3, 3), (5, 9)]):
        m, ids, cnt = F.scan(f, b, z, br, want_ids=True)
        om = oracle.z3filter_scan(F.serialize_to_bytes(f), br, b, z)
        assert np.array_equal(as_np(m), om) and cnt == int(om.sum())
    f2 = F.Z2Filter([[-2**31, -5, 2**31 - 1, 100], [10, 10, 5, 5], [0, 0, 1 << 20, 1 << 20],
                     [-(1 << 30), -(1 << 31), -1, -1]][: k + 2])
    m, ids, cnt = F.z2_scan(f2, z, want_ids=True)
    om = oracle.z2filter_scan(F.z2_serialize_to_bytes(f2), z)
    assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])


def test_filter_scan_many_boxes_generic_path(gpu, oracle):
    """More than 4 boxes / bin ranges takes the generic (descriptor-walking) kernel."""
    x, y, t = random_keys(200_003, seed=77)
    ks = Z3IndexKeySpace()
    b, z = ks.sfc.index_keys(x, y, t)
    boxes = [(-170 + 30 * i, -60, -160 + 30 * i, 60) for i in range(6)]
    v = ks.get_index_values(boxes, [during(ms("2020-02-01T00:00:00.000Z"), ms("2020-09-08T12:00:00.000Z"))])
    f = F.Z3Filter.from_values(v)
    br = [(2611, 2612), (2614, 2614), (2620, 2630), (2633, 2640), (2645, 2650)]
    m, ids, n = F.scan(f, b, z, br, want_ids=True)
    om = oracle.z3filter_scan(F.serialize_to_bytes(f), br, as_np(b), as_np(z))
    assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])


def test_filter_scan_empty(gpu):
    f = F.Z3Filter([[0, 0, 10, 10]], [], 32767, -32768)
    m, ids, n = F.scan(f, np.zeros(0, np.int16), np.zeros(0, np.int64), [], want_ids=True)
    assert n == 0 and m.numel() == 0


# ---------------------------------------------------------------- st_contains join
def test_st_contains_box_kats_gpu(gpu):  # geomesa-spark-jts/.../SpatialRelationFunctionsTest.scala:85-107
    from geomesa_amd.join import PolygonIndex, PolygonSet
    ps = PolygonSet.from_wkt(["POLYGON((0  0,  0 10, 10 10, 10  0,  0  0))"])
    pts = {"int": (5.0, 5.0), "edge": (0.0, 5.0), "corner": (0.0, 0.0), "ext": (-5.0, 0.0)}
    names = list(pts)
    pt, pl = PolygonIndex(ps).join([pts[k][0] for k in names], [pts[k][1] for k in names])
    assert [names[i] for i in as_np(pt)] == ["int"]


def test_st_contains_holes_multipolygon_gpu(gpu, oracle):
    from geomesa_amd.join import PolygonIndex, PolygonSet
    ps = PolygonSet.from_wkt([
        "POLYGON((0 0, 0 10, 10 10, 10 0, 0 0), (3 3, 6 3, 6 6, 3 6, 3 3))",
        "MULTIPOLYGON(((0 0, 0 10, 5 10, 5 0, 0 0)), ((5 0, 5 10, 10 10, 10 0, 5 0)))",
        "POLYGON((20 20, 25 30, 30 20, 25 25, 20 20))"])
    xs, ys = np.meshgrid(np.arange(-1, 31.0, 0.5), np.arange(-1, 31.0, 0.5))
    px, py = xs.ravel(), ys.ravel()
    pt, pl = PolygonIndex(ps).join(px, py)
    import oracle as O
    ops = O.OraclePolySet(*ps.to_arrays())
    opt, opl = ops.join(px, py)
    assert sorted(zip(as_np(pt).tolist(), as_np(pl).tolist())) == sorted(zip(opt.tolist(), opl.tolist()))
    got = set(zip(as_np(pt).tolist(), as_np(pl).tolist()))
    k = lambda x, y: int(np.nonzero((px == x) & (py == y))[0][0])  # noqa: E731
    assert (k(1, 1), 0) in got and (k(4, 4), 0) not in got and (k(3, 4), 0) not in got
    assert (k(5, 5), 1) in got  # shared component edge: Mod-2 -> interior


@pytest.mark.parametrize("grid,cells_per_poly", [((20, 10), 0), ((80, 40), 0), ((20, 10), 1), ((20, 10), 16),
                                                 ((20, 10), 4096)])
def test_pip_join_synthetic_counties(gpu, oracle, grid, cells_per_poly):
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(*grid)
    px, py = synthetic_points(400_000)
    # adversarial points: every vertex, segment midpoints, and points on cell lines
    vx, vy = ps.vx[::3], ps.vy[::3]
    px = np.concatenate([px, vx, (ps.vx[1:] + ps.vx[:-1]) / 2, np.full(1000, -95.5)])
    py = np.concatenate([py, vy, (ps.vy[1:] + ps.vy[:-1]) / 2, np.linspace(24, 50, 1000)])
    ix = PolygonIndex(ps, cells_per_poly=cells_per_poly)
    if cells_per_poly == 1:
        assert ix.stats()["slow"] > 0   # exercises the slab-walk fallback
    import oracle as O
    opt, opl = O.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=8)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    pt, pl = ix.join(px, py)
    assert np.array_equal(_sorted_pairs(pt, pl), exp)
    assert ix.join(px, py, count_only=True) == len(exp)
    # capacity path
    pt2, pl2 = ix.join(px, py, cap=10)
    assert len(pt2) == len(exp)


def _sorted_pairs(pt, pl):
    got = np.stack([as_np(pt), as_np(pl).astype(np.int64)], 1)
    return got[np.lexsort((got[:, 1], got[:, 0]))]


def test_pip_join_edges(gpu, oracle):
    """NaN / infinite / off-grid points never match, id_base offsets ids, empty and one-point input."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(20, 10)
    ix = PolygonIndex(ps)
    px, py = synthetic_points(300_000, seed=5)
    px[::97] = np.nan; py[::89] = np.nan
    py[::101] = 1e9; px[::103] = -1e9
    py[::107] = np.inf; px[::109] = -np.inf
    import oracle as O
    opt, opl = O.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=8)
    exp = np.stack([opt + 1000, opl.astype(np.int64)], 1)
    pt, pl = ix.join(px, py, id_base=1000)
    assert np.array_equal(_sorted_pairs(pt, pl), exp)
    assert ix.join(px[:0], py[:0])[0].numel() == 0
    assert ix.join(px[:1], py[:1], count_only=True) == int((opt == 0).sum())


def test_pip_join_unknown_mode_rejected(gpu):
    """Only GM_JOIN_AUTO / GM_JOIN_DIRECT exist (the band-partitioned and two-pass strategies were
    removed); any other mode is GM_E_INVALID through the C ABI, for columns and Arrow input alike."""
    import ctypes
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ix = PolygonIndex(synthetic_counties(4, 2))
    x = torch.full((16,), -100.0, dtype=torch.float64, device="cuda")
    npairs = ctypes.c_int64(-1)
    for mode in (2, 3, -1):
        rc = ix.ctx.lib.gm_pip_join_ex(ix.ctx.handle, ix._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                       16, 0, None, None, 0, ctypes.byref(npairs), mode)
        assert rc == _lib.GM_E_INVALID, mode
    for mode in (_lib.GM_JOIN_AUTO, _lib.GM_JOIN_DIRECT):
        rc = ix.ctx.lib.gm_pip_join_ex(ix.ctx.handle, ix._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                       16, 0, None, None, 0, ctypes.byref(npairs), mode)
        assert rc == _lib.GM_OK and npairs.value == 0


def test_pip_join_auto_large(gpu, oracle):
    """5M points x 3,200 polygons: auto and direct (the same staged pass) equal the oracle."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(80, 40)
    ix = PolygonIndex(ps)
    px, py = synthetic_points(5_000_000, seed=9)
    import oracle as O
    opt, opl = O.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=16)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    pt, pl = ix.join(px, py)
    assert np.array_equal(_sorted_pairs(pt, pl), exp)
    assert ix.join(px, py, count_only=True, mode="direct") == len(exp)
    pt, pl = ix.join(px, py, mode="direct", predicate="st_within")
    assert np.array_equal(_sorted_pairs(pt, pl), exp)


# ---------------------------------------------------------------- batched ranges
def test_z3_ranges_kats_gpu(gpu, oracle):  # geomesa-z3/src/test/.../curve/Z3Test.scala:182-220
    from test_oracle_kats import z3_test_boxes
    from geomesa_amd.curve import Z3SFC
    sfc = Z3SFC("week")
    # drive through ZN.zranges bounds directly: invert the corners back to user space boxes
    boxes = z3_test_boxes(oracle)
    for (lo, hi) in boxes[:16]:
        x0, y0, t0 = oracle.z3_invert(lo); x1, y1, t1 = oracle.z3_invert(hi)
        exp = oracle.z3_ranges([(x0, y0, x1, y1)], [(t0, t1)], max_ranges=1000)
        got = sfc.ranges([(x0, y0, x1, y1)], [(t0, t1)], max_ranges=1000)
        assert [tuple(r) for r in got] == exp and 0 < len(got) <= 1000


def ranges_queries(n, seed=13):
    rng = np.random.default_rng(seed)
    qs = []
    for _ in range(n):
        w = 10 ** rng.uniform(-2, 1.3); h = 10 ** rng.uniform(-2, 1.3)
        cx = rng.uniform(-180 + w, 180 - w); cy = rng.uniform(-90 + h, 90 - h)
        t0 = int(rng.integers(0, 604800)); t1 = int(min(604800, t0 + 10 ** rng.uniform(1, 5.8)))
        qs.append(((cx - w, cy - h, cx + w, cy + h), (t0, t1)))
    return qs


@pytest.mark.parametrize("max_ranges", [2000, 250, 7, 1, None])
def test_z3_ranges_batch_parity(gpu, oracle, max_ranges):
    from geomesa_amd.curve import Z3SFC
    qs = ranges_queries(40 if max_ranges is None else 300)
    if max_ranges is None:
        qs = [((b[0], b[1], b[0] + 0.001, b[1] + 0.001), (t[0], t[0] + 60)) for b, t in qs]
    got = Z3SFC("week").ranges_batch([([b], [t]) for b, t in qs], 64, max_ranges)
    for (b, t), g in zip(qs, got):
        exp = oracle.z3_ranges([b], [t], max_ranges=max_ranges)
        assert [tuple(r) for r in g] == exp


def test_z3_ranges_multi_bounds_and_precision(gpu, oracle):
    from geomesa_amd.curve import Z3SFC
    xy = [(-10, 35, 30, 60), (100, -40, 120, -10)]
    t = [(0, 3600), (86400, 90000), (500000, 604800)]
    for prec, mr in [(64, 2000), (40, 2000), (64, 50), (20, None)]:
        exp = oracle.z3_ranges(xy, t, precision=prec, max_ranges=mr)
        got = Z3SFC("week").ranges(xy, t, precision=prec, max_ranges=mr)
        assert [tuple(r) for r in got] == exp


@pytest.mark.parametrize("max_ranges", [1000, 100, None])
def test_z2_ranges_batch_parity(gpu, oracle, max_ranges):
    from geomesa_amd.curve import Z2SFC
    qs = [b for b, _ in ranges_queries(200, seed=17)]
    got = Z2SFC().ranges_batch([[b] for b in qs], 64, max_ranges)
    for b, g in zip(qs, got):
        assert [tuple(r) for r in g] == oracle.z2_ranges([b], max_ranges=max_ranges)


@pytest.mark.parametrize("max_ranges", [None, 2000, 100, 3])
def test_xz2_ranges_batch_parity(gpu, oracle, max_ranges):
    from geomesa_amd.curve import XZ2SFC
    qs = [[b] for b, _ in ranges_queries(150, seed=19)] + [[(45.0, 23.0, 48.0, 27.0)],
                                                           [(-180.0, -90.0, 180.0, 90.0)],
                                                           [(11.0, 11.0, 11.0, 11.0), (0.0, 0.0, 20.0, 20.0)]]
    got = XZ2SFC(12).ranges_batch(qs, max_ranges)
    for q, g in zip(qs, got):
        assert [tuple(r) for r in g] == oracle.xz2_ranges(q, max_ranges=max_ranges)


@pytest.mark.parametrize("dims", [2, 3])
@pytest.mark.parametrize("max_ranges", [1 << 28, 1 << 30, (1 << 31) - 1])
def test_xz_ranges_huge_budget(gpu, oracle, dims, max_ranges):
    """A maxRanges far past the workspace caps (a caller meaning "unlimited") runs with the unbounded
    caps instead of failing the call, and gives the oracle's lists."""
    from geomesa_amd.curve import XZ2SFC, XZ3SFC
    qs = [[b] for b, _ in ranges_queries(20, seed=71)] + [[(-180.0, -90.0, 180.0, 90.0)]]
    if dims == 3:
        qs = [[(b[0], b[1], 100.0, b[2], b[3], 5000.0)] for (b,) in qs]
    sfc = XZ2SFC(12) if dims == 2 else XZ3SFC(12, "week")
    got = sfc.ranges_batch(qs, max_ranges)
    for q, g in zip(qs, got):
        exp = oracle.xz2_ranges(q, max_ranges=max_ranges) if dims == 2 else oracle.xz3_ranges(q, max_ranges=max_ranges)
        assert [tuple(r) for r in g] == exp


@pytest.mark.parametrize("dims", [2, 3])
def test_xz_ranges_many_windows(gpu, oracle, dims):
    """Queries with more windows than the first pass stages in LDS (16) run again in the second pass
    with every window in LDS; batched with one-window queries, the output equals the oracle's."""
    from geomesa_amd.curve import XZ2SFC, XZ3SFC
    rng = np.random.default_rng(31 + dims)
    qs = []
    for k in range(40):
        nw = [1, 15, 16, 17, 40, 256][k % 6]
        ws = []
        for _ in range(nw):
            x0, y0 = rng.uniform(-170, 160), rng.uniform(-80, 70)
            w, h = rng.uniform(0.01, 8), rng.uniform(0.01, 8)
            if dims == 2:
                ws.append((x0, y0, x0 + w, y0 + h))
            else:
                t0 = rng.uniform(0, 500000)
                ws.append((x0, y0, t0, x0 + w, y0 + h, t0 + rng.uniform(60, 90000)))
        qs.append(ws)
    sfc = XZ2SFC(12) if dims == 2 else XZ3SFC(12, "week")
    got = sfc.ranges_batch(qs, 2000)
    for q, g in zip(qs, got):
        exp = oracle.xz2_ranges(q, max_ranges=2000) if dims == 2 else oracle.xz3_ranges(q, max_ranges=2000)
        assert [tuple(r) for r in g] == exp


@pytest.mark.parametrize("max_ranges", [10000, 2000, 50])
def test_xz3_ranges_batch_parity(gpu, oracle, max_ranges):
    from geomesa_amd.curve import XZ3SFC
    qs = [[(b[0], b[1], float(t[0]), b[2], b[3], float(t[1]))] for b, t in ranges_queries(60, seed=23)]
    qs.append([(45.0, 23.0, 900.0, 48.0, 27.0, 1100.0)])
    got = XZ3SFC(12, "week").ranges_batch(qs, max_ranges)
    for q, g in zip(qs, got):
        assert [tuple(r) for r in g] == oracle.xz3_ranges(q, max_ranges=max_ranges)


def test_xz2_kats_gpu(gpu):  # geomesa-z3/src/test/.../curve/XZ2SFCTest.scala:24-128
    from conftest import load_geoms
    from test_oracle_kats import CONTAINING, DISJOINT, OVERLAPPING
    from geomesa_amd.curve import XZ2SFC
    sfc = XZ2SFC(12)
    poly = int(as_np(sfc.index([10.0], [10.0], [12.0], [12.0]))[0])
    hit = lambda rs, v: any(r.lower <= v <= r.upper for r in rs)  # noqa: E731
    rs = sfc.ranges_batch([[b] for b in CONTAINING + OVERLAPPING + DISJOINT])
    assert all(hit(r, poly) for r in rs[:8]) and not any(hit(r, poly) for r in rs[8:])
    g = np.array(load_geoms())
    idx = as_np(sfc.index(g[:, 0], g[:, 1], g[:, 2], g[:, 3]))
    rr = sfc.ranges([(45.0, 23.0, 48.0, 27.0)])
    assert all(hit(rr, int(v)) for v in idx)


@pytest.mark.parametrize("kind", ["xz2", "xz3", "z3"])
def test_ranges_pipelined_chunks(gpu, oracle, kind):
    """Batched ranges into pinned host memory in pipelined query chunks (GM_PARAM_RANGES_CHUNK): the
    chunk results copied back on a second stream while the next chunk runs give exactly the
    one-batch offsets, ranges and statuses, also through a capacity retry (gm_ranges.hip run_ranges)."""
    import ctypes
    from geomesa_amd import _lib
    from geomesa_amd import ranges as R
    from geomesa_amd.curve import XZ2SFC, XZ3SFC, Z3SFC
    ctx = _lib.context()
    if kind == "z3":
        qs = [([b], [(int(t[0]), int(t[1]))]) for b, t in ranges_queries(70, seed=29)]
        fn, args, nq, cap = R.prepare_z3(Z3SFC("week"), qs, 64, 300)
    else:
        d = 2 if kind == "xz2" else 3
        sfc = XZ2SFC(12) if d == 2 else XZ3SFC(12, "week")
        qs = [[b] if d == 2 else [(b[0], b[1], float(t[0]), b[2], b[3], float(t[1]))]
              for b, t in ranges_queries(70, seed=31)]
        off, w = R._windows(qs, d)
        nq, cap = len(qs), len(qs) * 4096
        fn = ctx.lib.gm_xz2_ranges if d == 2 else ctx.lib.gm_xz3_ranges
        args = (ctx.handle, nq, off.ctypes.data, w.ctypes.data, 12, 300) if d == 2 else \
            (ctx.handle, nq, off.ctypes.data, w.ctypes.data, 12, sfc.period, 300)
    o1, r1, s1 = R.call_raw(fn, args, nq, cap)                       # pageable output: one batch
    r1 = r1[:int(o1[-1])].copy()
    try:
        for chunk in (1, 7, 64):
            ctx.set_param(_lib.GM_PARAM_RANGES_CHUNK, chunk)
            o2, r2, s2 = R.call_raw(fn, args, nq, cap, pinned=True)
            assert np.array_equal(o1, o2) and np.array_equal(s1, s2), chunk
            assert np.array_equal(r1, r2[:int(o2[-1])]), chunk
            # a capacity below the total: GM_E_CAPACITY with the exact need, then the retry
            o3, r3, _ = R.call_raw(fn, args, nq, max(1, int(o1[-1]) // 3), pinned=True)
            assert np.array_equal(o1, o3) and np.array_equal(r1, r3[:int(o3[-1])]), chunk
    finally:
        ctx.set_param(_lib.GM_PARAM_RANGES_CHUNK, 0)
    if kind == "xz2":   # and the oracle, for one query
        got = [(int(r["lower"]), int(r["upper"]), bool(r["contained"])) for r in r1[int(o1[0]):int(o1[1])]]
        assert got == [(int(a), int(b), bool(c)) for a, b, c in oracle.xz2_ranges(qs[0], max_ranges=300)]


@pytest.mark.parametrize("kind", ["z3", "xz2", "xz3"])
def test_ranges_device_output(gpu, kind):
    """Batched ranges written straight into device memory (ranges for a device-side consumer: no copy
    back) equal the host-output batch: offsets, ranges and statuses."""
    import ctypes
    import torch
    from geomesa_amd import _lib
    from geomesa_amd import ranges as R
    from geomesa_amd.curve import XZ3SFC, Z3SFC
    ctx = _lib.context()
    if kind == "z3":
        qs = [([b], [(int(t[0]), int(t[1]))]) for b, t in ranges_queries(50, seed=37)]
        fn, args, nq, cap = R.prepare_z3(Z3SFC("week"), qs, 64, 500)
    else:
        d = 2 if kind == "xz2" else 3
        qs = [[b] if d == 2 else [(b[0], b[1], float(t[0]), b[2], b[3], float(t[1]))]
              for b, t in ranges_queries(50, seed=41)]
        off, w = R._windows(qs, d)
        nq, cap = len(qs), len(qs) * 4096
        fn = ctx.lib.gm_xz2_ranges if d == 2 else ctx.lib.gm_xz3_ranges
        args = (ctx.handle, nq, off.ctypes.data, w.ctypes.data, 12, 500) if d == 2 else \
            (ctx.handle, nq, off.ctypes.data, w.ctypes.data, 12, XZ3SFC(12, "week").period, 500)
    o1, r1, s1 = R.call_raw(fn, args, nq, cap)
    total = int(o1[-1])
    dev = torch.empty(max(total, 1) * R.RANGE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    o2 = np.zeros(nq + 1, np.int64)
    s2 = np.zeros(nq, np.int32)
    need = ctypes.c_int64()
    _lib.check(fn(*args, o2.ctypes.data, dev.data_ptr(), max(total, 1), ctypes.byref(need), s2.ctypes.data), "ranges")
    assert np.array_equal(o1, o2) and np.array_equal(s1, s2) and need.value == total
    r2 = dev[:total * R.RANGE_DTYPE.itemsize].cpu().numpy().view(R.RANGE_DTYPE)
    assert np.array_equal(r1[:total], r2)
