"""GPU parity of the boundary entry points that take the reference's raw forms: ZN.zranges over raw
ZRange bounds (gm_zranges), RowFilter.inBounds over row-key bytes (gm_z3filter_scan_rows /
gm_z2filter_scan_rows), and the ZRange require failure of Appendix A.4."""
import numpy as np
import pytest

from test_gpu_scan_join_ranges import QUERIES, as_np, random_keys
from test_oracle_kats import z2_test_boxes, z3_test_boxes
from geomesa_amd import filters as F
from geomesa_amd.keyspace import Z2IndexKeySpace, Z3IndexKeySpace

pytestmark = pytest.mark.gpu


# ---------------------------------------------------------------- ZN.zranges on raw bounds
@pytest.mark.parametrize("legacy", [False, True])
def test_z3test_zranges_cases_gpu(gpu, oracle, legacy):
    """All 17 curve/Z3Test.scala:186-203 cases, including (z - 1, z + 1) ("62 bits in common"), through
    Z3.zranges(Array(ZRange(r._1, r._2)), maxRanges = Some(1000)) (:214) -- default maxRecurse 7."""
    from geomesa_amd.ranges import zranges
    boxes = z3_test_boxes(oracle, legacy)
    got = zranges(3, [[b] for b in boxes], max_ranges=1000)
    for b, g in zip(boxes, got):
        assert [tuple(r) for r in g] == oracle.zranges(3, [b], max_ranges=1000)
        assert 0 < len(g) <= 1000


@pytest.mark.parametrize("legacy", [False, True])
def test_z2test_zranges_cases_gpu(gpu, oracle, legacy):  # curve/Z2Test.scala:117-143
    from geomesa_amd.ranges import zranges
    boxes = z2_test_boxes(oracle, legacy)
    got = zranges(2, [[b] for b in boxes], max_ranges=1000)
    for b, g in zip(boxes, got):
        assert [tuple(r) for r in g] == oracle.zranges(2, [b], max_ranges=1000)
        assert 0 < len(g) <= 1000


def test_calculate_ranges_gpu(gpu, oracle):  # curve/Z3Test.scala:169-180, curve/Z2Test.scala:103-115
    from geomesa_amd.curve import CoveredRange
    from geomesa_amd.ranges import zranges
    Z = lambda x, y: oracle.z3_apply(x, y, 0)  # noqa: E731
    r3, = zranges(3, [[(Z(2, 2), Z(3, 6))]])
    assert sorted(r3) == sorted([CoveredRange(Z(2, 2), Z(3, 3)), CoveredRange(Z(2, 4), Z(3, 5)),
                                 CoveredRange(Z(2, 6), Z(3, 6))])
    Z2 = oracle.z2_apply
    r2, = zranges(2, [[(Z2(2, 2), Z2(3, 6))]])
    assert sorted(r2) == sorted([CoveredRange(Z2(2, 2), Z2(3, 3)), CoveredRange(Z2(2, 4), Z2(3, 5)),
                                 CoveredRange(Z2(2, 6), Z2(3, 6))])


@pytest.mark.parametrize("max_ranges,max_recurse", [(2000, None), (50, None), (None, 3), (7, 30), (1, None)])
def test_zranges_random_parity(gpu, oracle, max_ranges, max_recurse):
    """Random multi-bound queries (ZRange arrays of 1-3 bounds) against the oracle's ZN.zranges."""
    from geomesa_amd.ranges import zranges
    rng = np.random.default_rng(41)
    for dims in (2, 3):
        qs = []
        for _ in range(60):
            bounds = []
            for _ in range(int(rng.integers(1, 4))):
                a, b = sorted(int(v) for v in rng.integers(0, (1 << (21 * dims if dims == 3 else 62)) - 1, 2))
                if rng.random() < 0.5:   # narrow bound: long common prefix
                    b = a + int(rng.integers(0, 1 << 20))
                bounds.append((a, b))
            qs.append(bounds)
        got = zranges(dims, qs, max_ranges=max_ranges, max_recurse=max_recurse)
        for q, g in zip(qs, got):
            exp = oracle.zranges(dims, q, max_ranges=max_ranges, max_recurse=7 if max_recurse is None else max_recurse)
            assert [tuple(r) for r in g] == exp


def test_zranges_unordered_bound_gpu(gpu):
    from geomesa_amd.curve import IllegalArgumentException
    from geomesa_amd.ranges import zranges
    with pytest.raises(IllegalArgumentException, match="ordered"):
        zranges(3, [[(10, 5)]])


def test_ranges_wrapped_max_corner_gpu(gpu):  # SURVEY Appendix A.4, zorder/sfcurve/package.scala:24
    """Z3SFC.ranges with the max corner at nextafter(180, 0): normalize gives 2^21, Z3.split masks it
    to 0, index(min) > index(max) and the ZRange require throws."""
    from geomesa_amd.curve import IllegalArgumentException, Z3SFC
    x = float(np.nextafter(180.0, 0.0))
    with pytest.raises(IllegalArgumentException, match="ordered"):
        Z3SFC("week").ranges([(170.0, 0.0, x, 10.0)], [(0, 100)], 64, 2000)
    assert len(Z3SFC("week").ranges([(170.0, 0.0, 179.0, 10.0)], [(0, 100)], 64, 2000)) > 0


# ---------------------------------------------------------------- RowFilter.inBounds on row bytes
def _rows(keys, rng, shard=None):
    """Row-key bytes [shard?][bin][z] + a variable-length feature id, back to back, with offsets."""
    n = keys.shape[0]
    idl = rng.integers(0, 24, n)
    lens = keys.shape[1] + idl
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(lens)
    buf = np.empty(int(off[-1]), np.uint8)
    pos = np.repeat(off[:-1], keys.shape[1]) + np.tile(np.arange(keys.shape[1]), n)
    buf[pos] = keys.reshape(-1)
    fill = np.ones(int(off[-1]), bool)
    fill[pos] = False
    buf[fill] = rng.integers(0, 256, int(fill.sum()), dtype=np.uint8)
    return buf, off


@pytest.mark.parametrize("q", QUERIES)
@pytest.mark.parametrize("sharded", [False, True])
def test_z3filter_scan_rows_parity(gpu, oracle, q, sharded):
    """gm_z3filter_scan_rows over gm_z3_key_bytes output (with and without a shard byte, plus ragged
    feature ids) equals the oracle's Z3Filter.inBounds on the same keys."""
    import ctypes
    import torch
    from geomesa_amd import _lib
    x, y, t = random_keys(300_001, seed=3)
    ks = Z3IndexKeySpace()
    b, z = ks.sfc.index_keys(x, y, t)
    n = z.numel()
    ctx = _lib.context()
    shard = torch.from_numpy(np.arange(n, dtype=np.int64).astype(np.uint8) % 4).cuda() if sharded else None
    kl = 11 if sharded else 10
    kb = torch.empty(n * kl, dtype=torch.uint8, device=z.device)
    _lib.check(ctx.lib.gm_z3_key_bytes(ctx.handle, _lib.ptr(shard), _lib.ptr(b), _lib.ptr(z), n, _lib.ptr(kb)), "kb")
    rng = np.random.default_rng(5)
    buf, off = _rows(as_np(kb).reshape(n, kl), rng)
    v = ks.get_index_values(q[0], [q[1]])
    f = F.Z3Filter.from_values(v)
    fb = F.serialize_to_bytes(f)
    m, ids, k, short = F.scan_rows(f, buf, off, key_offset=kl - 10, want_ids=True)
    om = oracle.z3filter_scan(fb, [], as_np(b), as_np(z))
    assert short == 0 and k == int(om.sum())
    assert np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])
    for i in list(np.nonzero(om)[0][:20]) + list(range(20)):   # row-at-a-time against the oracle's inBounds
        assert bool(as_np(m)[i]) == oracle.z3filter_in_bounds(fb, bytes(buf[off[i]:off[i + 1]]), kl - 10)
    del ctypes


def test_filter_scan_rows_short_and_z2(gpu, oracle):
    """Z2Filter on row bytes, and rows too short for their key (counted, never matching)."""
    from geomesa_amd.curve import Z2SFC
    x, y, _ = random_keys(100_003, seed=8)
    z = as_np(Z2SFC().index(x, y))
    keys = z.astype(">i8").view(np.uint8).reshape(-1, 8)
    rng = np.random.default_rng(9)
    buf, off = _rows(keys, rng)
    f2 = F.Z2Filter.from_values(Z2IndexKeySpace().get_index_values([(-10, 35, 30, 60), (100, -40, 120, -10)]))
    m, ids, k, short = F.scan_rows(f2, buf, off, want_ids=True)
    om = oracle.z2filter_scan(F.z2_serialize_to_bytes(f2), z)
    assert short == 0 and np.array_equal(as_np(m), om) and np.array_equal(as_np(ids), np.nonzero(om)[0])
    # truncate every 7th row to 5 bytes: no match, counted
    lens = np.diff(off)
    lens[::7] = 5
    off2 = np.zeros_like(off)
    off2[1:] = np.cumsum(lens)
    buf2 = np.concatenate([buf[off[i]:off[i] + lens[i]] for i in range(len(lens))])
    m2, _, k2, short2 = F.scan_rows(f2, buf2, off2)
    exp = om.copy()
    exp[::7] = False
    assert short2 == len(lens[::7]) and np.array_equal(as_np(m2), exp) and k2 == int(exp.sum())
    # empty batch
    assert F.scan_rows(f2, b"", np.zeros(1, np.int64))[2:] == (0, 0)


def test_retired_param_is_accepted_noop(gpu):
    """GM_PARAM_INDEX_CORE_RETIRED (7): the round-5 ABI change keeps it for one release as a no-op."""
    from geomesa_amd import _lib
    gpu.set_param(7, 1)
    assert gpu.get_param(7) == 0
    assert gpu.lib.gm_ctx_set_param(gpu.handle, 10, 0) == _lib.GM_E_INVALID
