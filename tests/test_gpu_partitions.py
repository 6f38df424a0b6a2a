"""GPU: geomesa-fs Z2Scheme / XZ2Scheme through the HIP kernels (partition names bit-exact against the
oracle and the reference's PartitionSchemeTest names; bbox partition enumeration via the GPU ranges)."""
import numpy as np
import pytest

from test_partitions_kats import KAT_NAMES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,bits,n1,n2", KAT_NAMES)
def test_partition_names_kat(gpu, kind, bits, n1, n2):
    from geomesa_amd.partitions import XZ2Scheme, Z2Scheme
    s = (Z2Scheme if kind == "z2" else XZ2Scheme)(bits)
    assert s.partition_names([10.0, -75.0], [10.0, 38.0]) == [n1, n2]


@pytest.mark.parametrize("bits", [2, 8, 10, 20, 24])
def test_partition_names_random(gpu, oracle, bits):
    from geomesa_amd.partitions import XZ2Scheme, Z2Scheme
    rng = np.random.default_rng(bits)
    x = rng.uniform(-180, 180, 5001); y = rng.uniform(-90, 90, 5001)
    x[:4] = [-180, 180, 0, 179.99999999999997]; y[:4] = [-90, 90, 0, 89.99999999999999]
    w = rng.uniform(0, 3, 5001); h = rng.uniform(0, 3, 5001)
    xmax = np.minimum(x + w, 180.0); ymax = np.minimum(y + h, 90.0)
    z2 = Z2Scheme(bits).partition_names(x, y)
    xz = XZ2Scheme(bits).partition_names(x, y, xmax, ymax)
    fz, fx = Z2Scheme(bits).format, XZ2Scheme(bits).format
    for i in range(len(x)):
        assert z2[i] == fz % oracle.z2_index(x[i], y[i], precision=bits // 2)[1]
        assert xz[i] == fx % oracle.xz2_index(x[i], y[i], xmax[i], ymax[i], g=bits // 2)[1]


def test_partition_names_raise_out_of_bounds(gpu):
    from geomesa_amd.curve import IllegalArgumentException
    from geomesa_amd.partitions import Z2Scheme
    with pytest.raises(IllegalArgumentException):
        Z2Scheme(10).partition_names([181.0], [0.0])


@pytest.mark.parametrize("box,count", [((-180, -90, 180, 90), 4), ((-1, -1, 1, 1), 4), ((-10, 5, 10, 6), 2)])
def test_intersecting_partitions_2bit(gpu, box, count):  # PartitionSchemeTest.scala:189-203
    from geomesa_amd.partitions import Z2Scheme
    parts = Z2Scheme(2).intersecting_partitions([box])
    assert len(parts) == count and len(set(parts)) == count
    assert Z2Scheme(2).intersecting_partitions([]) is None


def test_covering_bounds_4bit(gpu):  # Z2Scheme.getCoveringFilter (Z2Scheme.scala:31-45)
    from geomesa_amd.partitions import Z2Scheme
    s = Z2Scheme(4)
    names = s.intersecting_partitions([(-180, -90, 180, 90)])
    assert sorted(names) == ["%02d" % i for i in range(16)]
    cells = [s.covering_bounds(n) for n in names]
    assert sum((c[2] - c[0]) * (c[3] - c[1]) for c in cells) == pytest.approx(360.0 * 180.0)
    top_right = [c for c in cells if c[2] == 180.0 and c[3] == 90.0]
    assert len(top_right) == 1 and top_right[0][4:] == (False, False)
