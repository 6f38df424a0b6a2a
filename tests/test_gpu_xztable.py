"""GPU parity for the Z2 / XZ2 / XZ3 index tables: bin-less key bytes and sort, XZ3 keys from envelope +
dtg columns, and the query path ranges -> seek -> filter (gm_table_scan) against full scans.

The XZ key spaces always apply the full filter (XZ2IndexKeySpace.scala:122-125, XZ3IndexKeySpace.scala:
247-250), so a query through the table must return exactly the features a full scan with the same filter
returns (oracle.envelope_scan: JTS Envelope.intersects + FastDuring, every feature) -- which also proves
the ranges cover every matching key.  The XZ2SFCTest / XZ3SFCTest geoms.list query (XZ2SFCTest.scala:
105-128) runs through the table: its seek returns all 135 envelopes."""
import numpy as np
import pytest

from conftest import load_geoms

pytestmark = pytest.mark.gpu

WEEK_MS = 604800000
T0 = 2600 * WEEK_MS          # 2019-11-07: bin 2600


def as_np(t):
    return t.detach().cpu().numpy()


def random_envelopes(n, seed, span=(0.0, 2.0)):
    """Envelopes of lines / polygons: centres uniform over the world, sizes log-uniform in span (degrees),
    some points (zero size) and a few world-spanning ones."""
    rng = np.random.default_rng(seed)
    cx, cy = rng.uniform(-180, 180, n), rng.uniform(-90, 90, n)
    w = np.exp(rng.uniform(np.log(1e-6), np.log(span[1] + 1e-6), n))
    h = np.exp(rng.uniform(np.log(1e-6), np.log(span[1] + 1e-6), n))
    w[rng.random(n) < 0.05] = 0.0
    h[rng.random(n) < 0.05] = 0.0
    big = rng.random(n) < 0.001
    w[big], h[big] = rng.uniform(30, 360, big.sum()), rng.uniform(20, 180, big.sum())
    xmin, xmax = np.clip(cx - w / 2, -180, 180), np.clip(cx + w / 2, -180, 180)
    ymin, ymax = np.clip(cy - h / 2, -90, 90), np.clip(cy + h / 2, -90, 90)
    return xmin, ymin, xmax, ymax


XZ_QUERIES = [
    [(-10.0, 35.0, 30.0, 60.0)],
    [(45.0, 23.0, 48.0, 27.0)],
    [(0.0, 0.0, 0.5, 0.5), (100.0, -40.0, 120.0, -10.0)],
    [(-180.0, -90.0, 180.0, 90.0)],
    [(179.0, 89.0, 180.0, 90.0)],
    None,                               # no spatial predicate: the whole world
]


@pytest.mark.parametrize("n", [1, 2049, 300_001])
@pytest.mark.parametrize("sharded", [False, True])
def test_sort_keys_without_bin(gpu, n, sharded):
    """gm_sort_keys with bin = NULL: the [shard][z BE64] order, stable."""
    import torch
    from geomesa_amd.table import _KeyTable
    rng = np.random.default_rng(n)
    z = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64, endpoint=True)
    z[rng.random(n) < 0.2] = 7
    sh = rng.integers(0, 4, n).astype(np.uint8) if sharded else None
    t = _KeyTable(None, z, sh)
    keys = [z.view(np.uint64)] + ([sh] if sharded else [])
    order = np.lexsort(keys)
    assert np.array_equal(as_np(t.perm), order) and np.array_equal(as_np(t.z), z[order])
    if sharded:
        assert np.array_equal(as_np(t.shard), sh[order])
    kb = as_np(t.key_bytes())
    exp = z[order].astype(">i8").view(np.uint8).reshape(n, 8)
    if sharded:
        exp = np.concatenate([sh[order].reshape(n, 1), exp], 1)
    assert np.array_equal(kb, exp)
    del torch


@pytest.mark.parametrize("lenient", [False, True])
def test_xz3_index_key_equals_binned_time_and_xz3(gpu, oracle, lenient):
    """gm_xz3_index_key = BinnedTime(dtg) then XZ3SFC.index at the offset (XZ3IndexKeySpace.scala:68-75),
    against the oracle's XZ3 index of the same envelopes at the same offsets; bad dates fail."""
    import ctypes
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.curve import _summary
    n = 200_003
    xmin, ymin, xmax, ymax = random_envelopes(n, 3)
    rng = np.random.default_rng(4)
    t = rng.integers(0, 60 * WEEK_MS, n) + T0
    t[:3] = [-1, 0, 32768 * WEEK_MS]                     # pre-1970 and past the max date: BAD_TIME
    cols = [torch.from_numpy(c).cuda() for c in (xmin, ymin, xmax, ymax)]
    tt = torch.from_numpy(t).cuda()
    b = torch.empty(n, dtype=torch.int16, device="cuda")
    xz = torch.empty(n, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    s = _summary()
    ctx = gpu
    _lib.check(ctx.lib.gm_xz3_index_key(ctx.handle, *[_lib.ptr(c) for c in cols], _lib.ptr(tt), n, 12, 1, int(lenient),
                                        _lib.ptr(b), _lib.ptr(xz), _lib.ptr(st), ctypes.byref(s)), "gm_xz3_index_key")
    st, b, xz = as_np(st), as_np(b), as_np(xz)
    assert s.n_errors == 2 and s.first_index == 0 and st[0] == _lib.GM_ST_BAD_TIME and st[2] == _lib.GM_ST_BAD_TIME
    assert st[1] == 0 and b[1] == 0
    ok = st == 0
    eb, eo = t // WEEK_MS, (t - t // WEEK_MS * WEEK_MS) // 1000
    assert np.array_equal(b[ok], eb[ok])
    env = np.stack([xmin, ymin, eo.astype(np.float64), xmax, ymax, eo.astype(np.float64)], 1)[ok]
    oz, ost = oracle.xz3_index_batch(env, lenient=lenient, g=12, period=oracle.WEEK)
    assert np.all(ost == 0) and np.array_equal(xz[ok], oz)
    assert np.all(b[~ok] == 0) and np.all(xz[~ok] == 0)


def test_xz2_table_geoms_list(gpu, oracle):
    """XZ2SFCTest "index complex features and query them2" (XZ2SFCTest.scala:105-128) through the table:
    the 135 envelopes of geoms.list ingested, the (45, 23, 48, 27) query's seek returns every one of them,
    and the full filter returns exactly the envelopes intersecting the box."""
    from geomesa_amd.table import XZ2Table
    g = np.array(load_geoms())
    assert len(g) == 135
    tb = XZ2Table(g[:, 0], g[:, 1], g[:, 2], g[:, 3], g=12)
    ids, n, scanned = tb.query([(45.0, 23.0, 48.0, 27.0)], full_filter=False)
    assert n == 135 and sorted(as_np(ids).tolist()) == list(range(135))
    ids, n, scanned = tb.query([(45.0, 23.0, 48.0, 27.0)])
    exp = np.nonzero(oracle.envelope_scan(g[:, 0], g[:, 1], g[:, 2], g[:, 3], [(45.0, 23.0, 48.0, 27.0)]))[0]
    assert np.array_equal(np.sort(as_np(ids)), exp) and scanned == 135


def test_xz3_table_geoms_list(gpu, oracle):
    """XZ3SFCTest.scala:105-128 through the table: every geoms.list envelope at t = 1000 s into a week,
    queried with (45, 23, 48, 27) during (900 s, 1100 s) of that week: all 135 come back."""
    from geomesa_amd.table import XZ3Table
    g = np.array(load_geoms())
    t = np.full(len(g), T0 + 1000_000, np.int64)
    tb = XZ3Table(g[:, 0], g[:, 1], g[:, 2], g[:, 3], t, g=12)
    ids, n, scanned = tb.query([(45.0, 23.0, 48.0, 27.0)], (T0 + 900_000, T0 + 1100_000), full_filter=False)
    assert n == 135 and sorted(as_np(ids).tolist()) == list(range(135))


@pytest.mark.parametrize("q", range(len(XZ_QUERIES)))
@pytest.mark.parametrize("sharded", [False, True])
def test_xz2_table_query_equals_full_scan(gpu, oracle, q, sharded):
    """ranges -> seek -> full filter over 1M envelopes equals the full filter over every envelope."""
    from geomesa_amd.table import XZ2Table
    n = 1_000_003
    xmin, ymin, xmax, ymax = random_envelopes(n, 10 + q)
    sh = (np.arange(n) * 2654435761 % 4).astype(np.uint8) if sharded else None
    tb = XZ2Table(xmin, ymin, xmax, ymax, shard=sh, shards=4 if sharded else None)
    boxes = XZ_QUERIES[q]
    ids, nm, scanned = tb.query(boxes)
    exp = np.nonzero(oracle.envelope_scan(xmin, ymin, xmax, ymax, boxes or [(-180.0, -90.0, 180.0, 90.0)]))[0]
    assert nm == len(exp) and np.array_equal(np.sort(as_np(ids)), exp)
    if q in (0, 1, 2, 4):
        assert scanned < n // 4   # the ranges prune


XZ3_QUERIES = [
    ([(-10.0, 35.0, 30.0, 60.0)], (T0 + 3 * WEEK_MS + 86_400_000, T0 + 3 * WEEK_MS + 5 * 86_400_000)),   # one bin
    ([(45.0, 23.0, 48.0, 27.0)], (T0 + WEEK_MS // 2, T0 + 9 * WEEK_MS // 2)),                            # 5 bins
    ([(0.0, 0.0, 2.0, 2.0), (100.0, -40.0, 120.0, -10.0)], (T0 + 1500, T0 + 2 * WEEK_MS + 999)),        # ms edges
    ([(-180.0, -90.0, 180.0, 90.0)], (T0 + 10 * WEEK_MS, T0 + 10 * WEEK_MS + 3_600_000)),
    ([(-50.0, -50.0, 50.0, 50.0)], None),                                                             # no dtg term
]


@pytest.mark.parametrize("q", range(len(XZ3_QUERIES)))
@pytest.mark.parametrize("sharded", [False, True])
def test_xz3_table_query_equals_full_scan(gpu, oracle, q, sharded):
    from geomesa_amd.table import XZ3Table
    n = 1_000_003
    xmin, ymin, xmax, ymax = random_envelopes(n, 20 + q)
    rng = np.random.default_rng(30 + q)
    t = T0 + rng.integers(0, 12 * WEEK_MS, n)
    t[:1000] = T0 + 1500 + np.arange(1000) % 3 - 1     # dtg exactly at / around the exclusive bounds
    sh = (np.arange(n) * 2654435761 % 4).astype(np.uint8) if sharded else None
    tb = XZ3Table(xmin, ymin, xmax, ymax, t, shard=sh, shards=4 if sharded else None)
    boxes, iv = XZ3_QUERIES[q]
    ids, nm, scanned = tb.query(boxes, iv)
    exp = np.nonzero(oracle.envelope_scan(xmin, ymin, xmax, ymax, boxes, t, iv))[0]
    assert nm == len(exp) and np.array_equal(np.sort(as_np(ids)), exp)
    if q in (0, 1, 2):
        assert scanned < n // 4


@pytest.mark.parametrize("strict", [False, True])
@pytest.mark.parametrize("sharded", [False, True])
def test_z2_table_query(gpu, oracle, strict, sharded):
    """Z2 point table: loose (Z2Filter on the row keys, the default) equals the oracle's Z2Filter over
    every key; strict (the full filter, point in bbox inclusive) equals a full scan of the points."""
    from geomesa_amd import filters as F
    from geomesa_amd.keyspace import Z2IndexKeySpace
    from geomesa_amd.table import Z2Table
    n = 1_000_003
    rng = np.random.default_rng(7)
    x, y = rng.uniform(-180, 180, n), rng.uniform(-90, 90, n)
    x[:100], y[:100] = 30.0, 60.0                              # exactly on a query corner
    sh = (np.arange(n) % 4).astype(np.uint8) if sharded else None
    tb = Z2Table(x, y, shard=sh, shards=4 if sharded else None)
    ks = Z2IndexKeySpace()
    for boxes in ([(-10.0, 35.0, 30.0, 60.0)], [(0.0, 0.0, 0.5, 0.5), (100.0, -40.0, 120.0, -10.0)]):
        ids, nm, scanned = tb.query(boxes, strict=strict)
        if strict:
            exp = np.nonzero(oracle.envelope_scan(x, y, x, y, boxes))[0]
        else:
            fb = F.serialize_to_bytes(F.Z2Filter.from_values(ks.get_index_values(boxes)))
            z = as_np(ks.sfc.index(x, y))
            exp = np.nonzero(oracle.z2filter_scan(fb, z))[0]
        assert nm == len(exp) and np.array_equal(np.sort(as_np(ids)), exp)
        assert scanned < n // 4


def test_table_scan_filter_errors(gpu):
    """gm_table_scan argument checks: both row filters, a Z3Filter without bins, boxes without columns."""
    import ctypes
    from geomesa_amd import _lib
    from geomesa_amd.table import _KeyTable, key_ranges
    tb = _KeyTable(None, np.arange(100, dtype=np.int64))
    arr, _ = key_ranges([("bounded", (0, 0), (0, 50))])
    f = _lib.ScanFilter()
    buf = ctypes.create_string_buffer(8)
    f.z3filter, f.z3filter_len, f.z2filter, f.z2filter_len = ctypes.addressof(buf), 8, ctypes.addressof(buf), 8
    with pytest.raises(_lib.GeomesaHipError):
        tb.table_scan(arr, f)
    f = _lib.ScanFilter()
    f.z3filter, f.z3filter_len = ctypes.addressof(buf), 8
    with pytest.raises(_lib.GeomesaHipError):
        tb.table_scan(arr, f)
    f = _lib.ScanFilter()
    f.n_boxes = 1
    with pytest.raises(_lib.GeomesaHipError):
        tb.table_scan(arr, f)
    ids, nm, ns = tb.table_scan(arr, None)
    assert nm == 51 and ns == 51 and sorted(as_np(ids).tolist()) == list(range(51))
