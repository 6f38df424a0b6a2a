"""GPU parity of the legacy curves (gm_legacy_*) against the C oracle, bit-exact (index and invert)."""
import numpy as np
import pytest

from test_gpu_parity import as_np, edge_points, f64_bits, random_points

pytestmark = pytest.mark.gpu


def _pts():
    x, y, t = random_points(20_001)
    ex, ey, et = edge_points()
    return np.concatenate([x, ex]), np.concatenate([y, ey]), np.concatenate([t % 700_000, et])


@pytest.mark.parametrize("period", [0, 1, 2, 3])
@pytest.mark.parametrize("lenient", [False, True])
def test_legacy_z3_index_invert(gpu, oracle, period, lenient):
    from geomesa_amd.curve import LegacyZ3SFC
    x, y, t = _pts()
    z, s = LegacyZ3SFC(period).index(x, y, t, lenient=lenient, status=True)
    z, s = as_np(z), as_np(s)
    for i in range(len(x)):
        st, oz = oracle.legacy_z3_index(float(x[i]), float(y[i]), int(t[i]), lenient, period)
        assert (s[i], z[i]) == (st, oz), i
    ok = s == 0
    xi, yi, ti = LegacyZ3SFC(period).invert(z[ok])
    ref = [oracle.legacy_z3_invert(int(v), period) for v in z[ok]]
    assert np.array_equal(f64_bits(as_np(xi)), f64_bits([r[0] for r in ref]))
    assert np.array_equal(f64_bits(as_np(yi)), f64_bits([r[1] for r in ref]))
    assert np.array_equal(as_np(ti), np.array([r[2] for r in ref], np.int64))


@pytest.mark.parametrize("lenient", [False, True])
def test_legacy_year_z3_index(gpu, oracle, lenient):
    from geomesa_amd.curve import LegacyYearZ3SFC
    x, y, t = _pts()
    t = np.concatenate([t[:-40], np.array([524160, 524161, 527050, 527051] * 10, np.int64)])
    z, s = LegacyYearZ3SFC().index(x, y, t, lenient=lenient, status=True)
    z, s = as_np(z), as_np(s)
    for i in range(len(x)):
        assert (s[i], z[i]) == oracle.legacy_year_z3_index(float(x[i]), float(y[i]), int(t[i]), lenient), i


@pytest.mark.parametrize("lenient", [False, True])
def test_legacy_z2_index_invert(gpu, oracle, lenient):
    from geomesa_amd.curve import IllegalArgumentException, LegacyZ2SFC
    x, y, _ = _pts()
    z, s = LegacyZ2SFC().index(x, y, lenient=lenient, status=True)
    z, s = as_np(z), as_np(s)
    for i in range(len(x)):
        assert (s[i], z[i]) == oracle.legacy_z2_index(float(x[i]), float(y[i]), lenient), i
    xi, yi = LegacyZ2SFC().invert(z[s == 0])
    ref = [oracle.legacy_z2_invert(int(v)) for v in z[s == 0]]
    assert np.array_equal(f64_bits(as_np(xi)), f64_bits([r[0] for r in ref]))
    assert np.array_equal(f64_bits(as_np(yi)), f64_bits([r[1] for r in ref]))
    with pytest.raises(IllegalArgumentException):
        LegacyZ2SFC().index([181.0], [0.0])


def test_z3_iterator_13_golden_gpu(gpu):
    """Z3IteratorTest.scala:82-93 on the device: gm_legacy_z3_index of the Z3IndexKeySpaceV4 query's
    corners decodes to the 1.3 install's golden option strings."""
    from geomesa_amd.curve import LegacyZ3SFC
    from geomesa_amd.keyspace import Z3IndexKeySpaceV4
    from test_host_planning import COMPAT_13_FILTER, COMPAT_13_GOLDEN, z3_dims
    v = Z3IndexKeySpaceV4().get_index_values(*COMPAT_13_FILTER)
    (xmin, ymin, xmax, ymax), = v.spatialBounds
    (t1, t2), = v.temporalBounds[2370]
    z = as_np(LegacyZ3SFC("week").index([xmin, xmax], [ymin, ymax], [t1, t2]))
    lo, hi = z3_dims(int(z[0])), z3_dims(int(z[1]))
    assert "%d:%d:%d:%d" % (lo[0], lo[1], hi[0], hi[1]) == COMPAT_13_GOLDEN["zxy"]
    assert "2370;%d:%d" % (lo[2], hi[2]) == COMPAT_13_GOLDEN["zt"]


@pytest.mark.parametrize("target", [2000, 250, 40])
def test_key_space_v4_ranges_and_keys(gpu, oracle, target):
    """Z3IndexKeySpaceV4 query planning over LegacyZ3SFC (legacy/Z3IndexV4.scala:44-51): getRanges runs
    Z3SFC.ranges as LegacyZ3SFC inherits it (Z3SFC.scala:59-67) -- ZRanges of the legacy index of each
    (box, interval)'s corners, Z3.zranges with Int.MaxValue recursion -- and toIndexKey is BinnedTime +
    the legacy index.  Checked against the oracle's legacy index and ZN.zranges."""
    from geomesa_amd.keyspace import Z3IndexKeySpaceV4
    from test_host_planning import COMPAT_13_FILTER
    ks = Z3IndexKeySpaceV4()
    v = ks.get_index_values(*COMPAT_13_FILTER)
    (xmin, ymin, xmax, ymax), = v.spatialBounds
    got = ks.sfc.ranges_batch([(v.spatialBounds, v.temporalBounds[b]) for b in sorted(v.temporalBounds)], 64, target)
    for b, rr in zip(sorted(v.temporalBounds), got):
        bounds = []
        for (t1, t2) in v.temporalBounds[b]:
            s0, lo = oracle.legacy_z3_index(xmin, ymin, int(t1))
            s1, hi = oracle.legacy_z3_index(xmax, ymax, int(t2))
            assert s0 == 0 and s1 == 0
            bounds.append((lo, hi))
        exp = oracle.zranges(3, bounds, 64, target, None)
        assert [(r.lower, r.upper, r.contained) for r in rr] == exp
    # get_ranges goes through the same call: [bin][z] ranges, one per IndexRange
    assert len(ks.get_ranges(v)) == sum(len(r) for r in ks.sfc.ranges_batch(
        [(v.spatialBounds, v.temporalBounds[b]) for b in sorted(v.temporalBounds)], 64, 2000 // len(v.temporalBounds)))
    # toIndexKey: BinnedTime(week) + LegacyZ3SFC.index
    x, y, t = random_points(5_001)
    bins, z = ks.to_index_keys(x, y, t)
    bins, z = as_np(bins), as_np(z)
    for i in range(0, len(x), 97):
        _, ob, off = oracle.binned_time(1, int(t[i]))
        st, oz = oracle.legacy_z3_index(float(x[i]), float(y[i]), int(off))
        assert (bins[i], z[i]) == (ob, oz), i
