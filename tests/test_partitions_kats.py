"""geomesa-fs Z2Scheme / XZ2Scheme partition names and bbox partition enumeration, pinned by the
reference's PartitionSchemeTest (geomesa-fs/geomesa-fs-storage/geomesa-fs-storage-common/src/test/
scala/org/locationtech/geomesa/fs/storage/common/partitions/PartitionSchemeTest.scala). CPU only:
the C oracle at the scheme's curve resolution."""
import numpy as np
import pytest

from geomesa_amd.curve import IllegalArgumentException
from geomesa_amd.partitions import XZ2Scheme, Z2Scheme

# PartitionSchemeTest.scala:97-146: POINT (10 10) and POINT (-75 38) (the date part of the composite
# scheme, "2017/003/", is not on this path)
KAT_NAMES = [
    ("z2", 10, "0770", "0617"), ("xz2", 10, "1030", "0825"),
    ("z2", 20, "0789456", "0632516"), ("xz2", 20, "1052614", "0843360"),
]


@pytest.mark.parametrize("kind,bits,n1,n2", KAT_NAMES)
def test_partition_name_kats(oracle, kind, bits, n1, n2):
    scheme = (Z2Scheme if kind == "z2" else XZ2Scheme)(bits)
    names = []
    for x, y in [(10.0, 10.0), (-75.0, 38.0)]:
        if kind == "z2":
            st, v = oracle.z2_index(x, y, precision=bits // 2)
        else:
            st, v = oracle.xz2_index(x, y, x, y, g=bits // 2)
        assert st == 0
        names.append(scheme.format % v)
    assert names == [n1, n2]


def test_scheme_digits_and_pattern():
    assert Z2Scheme(10).format == "%04d" and XZ2Scheme(10).format == "%04d"
    assert Z2Scheme(20).format == "%07d" and XZ2Scheme(20).format == "%07d"
    assert Z2Scheme(2).pattern == "2-bit-z2" and XZ2Scheme(4).pattern == "4-bit-xz2"
    with pytest.raises(IllegalArgumentException):
        Z2Scheme(3)


@pytest.mark.parametrize("box,count", [((-180, -90, 180, 90), 4), ((-1, -1, 1, 1), 4), ((-10, 5, 10, 6), 2),
                                       ((-179, -89, 179, 89), 4)])
def test_z2_2bit_partition_counts(oracle, box, count):  # PartitionSchemeTest.scala:160-203
    a = np.asarray(box, np.float64)
    rs = oracle._ranges_call(oracle.lib().gmo_z2_ranges, 1, oracle._p(a), 1, 64, 2147483647)
    parts = {v for r in rs for v in range(int(r[0]), int(r[1]) + 1)}
    assert len(parts) == count
