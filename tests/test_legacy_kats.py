"""Legacy curves (LegacyZ3SFC / LegacyZ2SFC / LegacyYearZ3SFC): the C oracle against the reference's own
tests that run them (z3t = geomesa-z3/src/test/scala/org/locationtech/geomesa/): curve/Z3Test.scala:49-75,
182-220 and curve/Z2Test.scala:48-64,117-143 iterate `Seq(Z3SFC(Week), LegacyZ3SFC(Week))` /
`Seq(Z2SFC, LegacyZ2SFC)`.  CPU only."""
import pytest

WEEK = 1
WEEK_S = 604800


def test_legacy_z3_max_values(oracle):  # Z3Test.scala:49-59: Z3(maxIndex...) round-trips
    for v in [(2**21 - 1, 2**21 - 1, 2**20 - 1)]:
        z = oracle.z3_apply(*v)
        assert (oracle.z3_combine(z), oracle.z3_combine(z >> 1), oracle.z3_combine(z >> 2)) == v
    st, z = oracle.legacy_z3_index(180.0, 90.0, WEEK_S)
    assert st == 0 and (oracle.z3_combine(z), oracle.z3_combine(z >> 1), oracle.z3_combine(z >> 2)) == \
        (2**21 - 1, 2**21 - 1, 2**20 - 1)


@pytest.mark.parametrize("x,y,t", [(-180.1, 0, 0), (180.1, 0, 0), (0, -90.1, 0), (0, 90.1, 0), (0, 0, -1),
                                   (0, 0, WEEK_S + 1), (-181, -91, -1), (181, 91, WEEK_S + 1)])
def test_legacy_z3_out_of_bounds(oracle, x, y, t):  # Z3Test.scala:61-75
    assert oracle.legacy_z3_index(float(x), float(y), t)[0] == 1
    assert oracle.legacy_z3_index(float(x), float(y), t, lenient=True)[0] == 0


@pytest.mark.parametrize("x,y", [(-180.1, 0), (0, -90.1), (180.1, 0), (0, 90.1), (-181, -91), (181, 91)])
def test_legacy_z2_out_of_bounds(oracle, x, y):  # Z2Test.scala:58-64
    assert oracle.legacy_z2_index(float(x), float(y))[0] == 1


def test_legacy_z3_ranges_ordered(oracle):  # Z3Test.scala:182-200: index(min corner) <= index(max corner)
    week, day, hour = WEEK_S, WEEK_S // 7, WEEK_S // 168
    cases = [((-180, -90, 0), (180, 90, week)), ((-180, -90, day), (180, 90, day * 2)),
             ((-180, -90, hour * 10), (180, 90, hour * 11)), ((-90, -45, week // 4), (90, 45, 3 * week // 4)),
             ((35, 65, 0), (45, 75, day)), ((35, 55, day), (45, 75, day * 2))]
    for lo, hi in cases:
        a = oracle.legacy_z3_index(float(lo[0]), float(lo[1]), lo[2])[1]
        b = oracle.legacy_z3_index(float(hi[0]), float(hi[1]), hi[2])[1]
        assert a <= b


def test_legacy_semantics(oracle):
    # SemiNormalizedDimension: the minimum maps to 0 and denormalizes to min exactly; ceil puts an
    # interior point in cell ceil(...), whose centre is within half a cell
    st, z = oracle.legacy_z2_index(-180.0, -90.0)
    assert st == 0 and z == 0 and oracle.legacy_z2_invert(0) == (-180.0, -90.0)
    st, z = oracle.legacy_z3_index(10.0, 20.0, 3600)
    x, y, t = oracle.legacy_z3_invert(z)
    assert abs(x - 10.0) <= 360.0 / (2**21 - 1) and abs(y - 20.0) <= 180.0 / (2**21 - 1)
    assert abs(t - 3600) <= WEEK_S / (2**20 - 1) + 1
    # legacy lenient clamps only from below: 181 -> ceil beyond maxIndex, masked by Z3.apply
    st, z = oracle.legacy_z3_index(181.0, 0.0, 0, lenient=True)
    assert st == 0
    # LegacyYearZ3SFC: offsets between 52 weeks and maxOffset(Year) index as the 52-week max
    m52 = 7 * 24 * 60 * 52
    assert oracle.legacy_year_z3_index(0.0, 0.0, m52 + 100)[1] == oracle.legacy_year_z3_index(0.0, 0.0, m52)[1]
    assert oracle.legacy_year_z3_index(0.0, 0.0, 527050)[0] == 0  # maxOffset(Year) = 1440 * 366 + 10
    assert oracle.legacy_year_z3_index(0.0, 0.0, 527051)[0] == 1
