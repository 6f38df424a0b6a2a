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
