"""Host-side logic (no GPU): query planning, Z3Filter wire formats, key layout, polygon CSR.

End-to-end known-answer tests run the reference query pipeline with the C oracle standing in for
the per-row work, pinning the planning code (interval rounding, epoch bins, filter construction)
to the reference's own expected result sets.
"""
import datetime
import struct

import numpy as np
import pytest

from geomesa_amd import filters as F
from geomesa_amd.keyspace import Bounds, Z3IndexKeySpace, between, during, extract_interval

UTC = datetime.timezone.utc


def ms(s):
    d = datetime.datetime.fromisoformat(s.replace("Z", "+00:00"))
    return int(round(d.timestamp() * 1000))


# ---------------------------------------------------------------- FilterHelperTest.scala
def test_interval_rounding():  # geomesa-filter/src/test/.../FilterHelperTest.scala:140-229
    a, b = ms("2016-01-01T00:00:00.000Z"), ms("2016-01-02T00:00:00.000Z")
    # no rounding without handleExclusiveBounds
    assert extract_interval(during(a, b), False) == Bounds(a, b, False, False)
    assert extract_interval(between(a, b), False) == Bounds(a, b, True, True)
    # narrow during stays exclusive (:150-154)
    assert extract_interval(during(a, a + 1000), True) == Bounds(a, a + 1000, False, False)
    # during rounds to [+1 s, -1 s] (:156-165)
    assert extract_interval(during(a, b), True) == Bounds(ms("2016-01-01T00:00:01.000Z"),
                                                          ms("2016-01-01T23:59:59.000Z"), True, True)
    assert extract_interval(between(a, b), True) == Bounds(a, b, True, True)
    # after / before with exclusive bounds (:192-203, :218-229)
    assert extract_interval(Bounds(a, None, False, True), True) == Bounds(ms("2016-01-01T00:00:01.000Z"), None,
                                                                        True, True)
    assert extract_interval(Bounds(ms("2016-01-01T00:00:01.000Z"), None, True, True), True).lower == \
        ms("2016-01-01T00:00:01.000Z")
    assert extract_interval(Bounds(None, a + 1, True, False), True) == Bounds(None, a, True, True)
    assert extract_interval(Bounds(None, a, True, True), True) == Bounds(None, a, True, True)


# ---------------------------------------------------------------- Z3FilterTest.scala
QUERIES = [  # geomesa-index-api/src/test/.../filters/Z3FilterTest.scala:28-32
    ([(38, 48, 52, 62)], [during(ms("2014-01-01T00:00:00.000Z"), ms("2014-01-08T12:00:00.000Z"))]),
    ([(38, 48, 52, 62)], [during(ms("2013-12-15T00:00:00.000Z"), ms("2014-01-15T00:00:00.000Z"))]),
    (None, [during(ms("2014-01-01T00:00:00.000Z"), ms("2014-01-08T12:00:00.000Z"))]),
]


@pytest.mark.parametrize("q", QUERIES)
def test_z3filter_serialization_round_trip(q):  # Z3FilterTest.scala:42-56
    ks = Z3IndexKeySpace()
    f = F.Z3Filter.from_values(ks.get_index_values(*q))
    assert F.deserialize_from_bytes(F.serialize_to_bytes(f)) == f
    assert F.deserialize_from_strings(F.serialize_to_strings(f)) == f


def test_z3filter_byte_layout():  # Z3Filter.scala:112-137 (big-endian, null epoch = -1)
    f = F.Z3Filter([[1, 2, 3, 4]], [[[5, 6]], None, [[7, 8], [9, 10]]], 100, 102)
    b = F.serialize_to_bytes(f)
    assert b == struct.pack(">i4ii i2i i i2i2i hh".replace(" ", ""), 1, 1, 2, 3, 4, 3, 1, 5, 6, -1, 2, 7, 8, 9, 10,
                            100, 102)
    s = F.serialize_to_strings(f)
    assert s["zxy"] == "1:2:3:4" and s["zt"] == "5:6,,7:8;9:10" and s["epoch"] == "100:102"


COMPAT_13_FILTER = ([(0, -70, 50, -50)], [during(ms("2015-06-06T00:00:00.000Z"), ms("2015-06-08T00:00:00.000Z"))])
# expected values "taken from a 1.3 install" (geomesa-accumulo/.../iterators/Z3IteratorTest.scala:90-92)
COMPAT_13_GOLDEN = {"zl": "8", "zo": "2", "zxy": "1048576:233017:1339847:466034", "zt": "2370;299595:599184"}


def z3_dims(z):
    """Z3(z).decode: the three 21-bit components (zorder/sfcurve/Z3.scala:83-91)."""
    return tuple(sum(((z >> (3 * i + d)) & 1) << i for i in range(21)) for d in range(3))


def test_z3_iterator_13_golden():  # Z3IteratorTest.scala:82-93: Z3IndexKeySpaceV4 -> LegacyZ3SFC(week)
    from geomesa_amd.keyspace import Z3IndexKeySpaceV4
    v = Z3IndexKeySpaceV4().get_index_values(*COMPAT_13_FILTER)
    assert F.z3_iterator_options(v, 2, "1.3") == COMPAT_13_GOLDEN
    with pytest.raises(NotImplementedError):
        F.z3_iterator_options(v, 2, "1.2")


def test_z3_iterator_13_golden_oracle(oracle):
    """The same strings from the C restatement's LegacyZ3SFC.index (gmo_legacy_z3_index) of the
    query corners, decoded: pins the oracle's semi-normalized dimensions to the 1.3 golden."""
    from geomesa_amd.keyspace import Z3IndexKeySpaceV4
    v = Z3IndexKeySpaceV4().get_index_values(*COMPAT_13_FILTER)
    (xmin, ymin, xmax, ymax), = v.spatialBounds
    (t1, t2), = v.temporalBounds[2370]
    lo = z3_dims(oracle.legacy_z3_index(xmin, ymin, t1)[1])
    hi = z3_dims(oracle.legacy_z3_index(xmax, ymax, t2)[1])
    assert "%d:%d:%d:%d" % (lo[0], lo[1], hi[0], hi[1]) == COMPAT_13_GOLDEN["zxy"]
    assert "2370;%d:%d" % (lo[2], hi[2]) == COMPAT_13_GOLDEN["zt"]


def test_z3_iterator_compat_values():  # Z3IteratorTest.scala:82-93's query through the MODERN curve
    # derived by restatement, not a reference golden: the golden above is the
    # legacy curve's; these pin only that the modern Z3Filter differs from it as expected
    ks = Z3IndexKeySpace()
    v = ks.get_index_values([(0, -70, 50, -50)], [during(ms("2015-06-06T00:00:00.000Z"),
                                                           ms("2015-06-08T00:00:00.000Z"))])
    assert list(v.temporalBounds) == [2370]
    assert v.temporalBounds[2370] == [(172801, 345599)]
    f = F.Z3Filter.from_values(v)
    s = F.serialize_to_strings(f)
    assert s["zxy"] == "1048576:233016:1339847:466033"   # derived for the modern curve (not pinned)
    assert s["zt"] == "599189:1198369" and s["epoch"] == "2370:2370"
    opts = F.z3_iterator_options(v, 0)   # compatibility None: the filter's strings + the row offset
    assert opts["zo"] == "0" and opts["zxy"] == s["zxy"]


# ---------------------------------------------------------------- key layout
def test_key_bytes():  # Z3IndexKeySpace.scala:81-92, ByteArrays.writeShort/writeLong
    kb = Z3IndexKeySpace.key_bytes(np.array([2370, -2], np.int16), np.array([0x0102030405060708, -1], np.int64))
    assert bytes(kb[0]) == b"\x09\x42\x01\x02\x03\x04\x05\x06\x07\x08"
    assert bytes(kb[1]) == b"\xff\xfe" + b"\xff" * 8
    kb = Z3IndexKeySpace.key_bytes(np.array([1], np.int16), np.array([2], np.int64), shard=np.array([3]))
    assert bytes(kb[0]) == b"\x03\x00\x01" + b"\x00" * 7 + b"\x02"


# ---------------------------------------------------------------- end-to-end KATs through the oracle
def idx_strategy_features():
    """Z3IdxStrategyTest.scala:39-64: 30 deterministic points."""
    feats = []
    for i in range(10):
        feats.append((i, 40.0 + i, 60.0, ms("2010-05-07T0%d:00:00.000Z" % i)))
    for i in range(10, 20):
        feats.append((i, 40.0 + (i - 10), 60.0, ms("2010-05-%dT%d:00:00.000Z" % (i, i))))
    for i in range(20, 30):
        feats.append((i, 60.0 + (i - 20), 60.0, ms("2010-05-%dT%02d:00:00.000Z" % (i, i - 10))))
    return feats


IDX_STRATEGY_KATS = [  # Z3IdxStrategyTest.scala:96-181
    ((38, 59, 51, 61), between(ms("2010-05-07T00:00:00.000Z"), ms("2010-05-08T00:00:00.000Z")), set(range(0, 10))),
    ((38, 59, 45, 61), between(ms("2010-05-07T00:00:00.000Z"), ms("2010-05-08T00:00:00.000Z")), set(range(0, 6))),
    ((38, 59, 51, 61), between(ms("2010-05-07T06:00:00.000Z"), ms("2010-05-08T00:00:00.000Z")), set(range(6, 10))),
    ((-180, -90, 180, 90), between(ms("2010-05-07T05:00:00.000Z"), ms("2010-05-07T08:00:00.000Z")), set(range(5, 9))),
    ((45, 59, 51, 61), between(ms("2010-05-07T06:00:00.000Z"), ms("2010-05-21T00:00:00.000Z")),
     set(range(6, 10)) | set(range(15, 20))),
    ((44.5, 59, 50, 61), between(ms("2010-05-10T00:00:00.000Z"), ms("2010-05-17T23:59:59.999Z")), set(range(15, 18))),
    ((-180, -90, 180, 90), between(ms("2010-05-07T06:00:00.000Z"), ms("2010-05-21T00:00:00.000Z")), set(range(6, 21))),
    ((-180, -90, 180, 90), between(ms("2010-05-08T06:00:00.000Z"), ms("2010-05-30T00:00:00.000Z")),
     set(range(10, 30))),
    ((40.999, 59.999, 41.001, 60.001), between(ms("2010-05-07T00:59:00.000Z"), ms("2010-05-07T01:01:00.000Z")), {1}),
    ((38, 59, 51, 61), Bounds(ms("2010-05-07T06:00:00.000Z"), ms("2010-05-08T00:00:00.000Z"), True, True),
     set(range(6, 10))),
]


def run_query_oracle(oracle, ks, feats, bbox, interval):
    ids = np.array([f[0] for f in feats])
    x = np.array([f[1] for f in feats]); y = np.array([f[2] for f in feats]); t = np.array([f[3] for f in feats])
    b, z, st = oracle.z3_index_key_batch(x, y, t)
    assert (st == 0).all()
    v = ks.get_index_values([bbox], [interval])
    fb = F.serialize_to_bytes(F.Z3Filter.from_values(v))
    m = oracle.z3filter_scan(fb, ks.bin_ranges(v), b, z)
    return set(ids[m].tolist())


@pytest.mark.parametrize("bbox,interval,expected", IDX_STRATEGY_KATS)
def test_idx_strategy_kats(oracle, bbox, interval, expected):
    ks = Z3IndexKeySpace()
    assert run_query_oracle(oracle, ks, idx_strategy_features(), bbox, interval) == expected


def test_z3_iterator_keep_drop(oracle):  # Z3IteratorTest.scala:64-80
    ks = Z3IndexKeySpace()
    v = ks.get_index_values([(-78, 38, -75, 40)], [during(ms("1970-01-01T00:05:00.000Z"),
                                                           ms("1970-01-01T00:15:00.000Z"))])
    fb = F.serialize_to_bytes(F.Z3Filter.from_values(v))
    keep = oracle.z3_index(-76.0, 38.5, 500)[1]
    drop = oracle.z3_index(-70.0, 38.5, 500)[1]
    assert oracle.z3filter_in_bounds(fb, b"\x00\x00" + struct.pack(">q", keep))
    assert not oracle.z3filter_in_bounds(fb, b"\x00\x00" + struct.pack(">q", drop))


def test_loose_vs_strict_bbox(oracle):  # geomesa-accumulo/.../data/AccumuloDataStoreQueryTest.scala:56,575-684
    x, y, t = np.array([45.0]), np.array([49.0]), np.array([ms("2010-05-07T12:30:00.000Z")])
    bbox = (45.000000001, 49.000000001, 46, 50)
    iv = during(ms("2010-05-07T12:25:00.000Z"), ms("2010-05-07T12:35:00.000Z"))
    ks = Z3IndexKeySpace()
    b, z, _ = oracle.z3_index_key_batch(x, y, t)
    v = ks.get_index_values([bbox], [iv])
    loose = oracle.z3filter_scan(F.serialize_to_bytes(F.Z3Filter.from_values(v)), ks.bin_ranges(v), b, z)
    assert loose[0]                                      # same normalized cell: returned (loose default)
    assert not oracle.strict_scan(x, y, t, bbox, (iv.lower, iv.upper))[0]   # strict BBOX drops it
    # Z2 loose
    z2, _ = oracle.z2_index_batch(x, y)
    from geomesa_amd.keyspace import Z2IndexKeySpace
    f2 = F.Z2Filter.from_values(Z2IndexKeySpace().get_index_values([bbox]))
    assert oracle.z2filter_scan(F.z2_serialize_to_bytes(f2), z2)[0]


def test_index_result_set_yearly(oracle):  # geomesa-index-api/src/test/.../index/Z3IndexTest.scala:26-64
    feats = []
    for i in range(10):
        feats.append((i, 40.0 + i, 60.0, ms("2020-12-07T0%d:00:00.000Z" % i)))
    for i in range(10, 20):
        feats.append((i, 40.0 + i - 10, 60.0, ms("2020-12-%dT%d:00:00.000Z" % (i, i))))
    for i in range(20, 30):
        feats.append((i, 60.0 + i - 20, 60.0, ms("2020-12-%dT%02d:00:00.000Z" % (i, i - 10))))
    for i in range(30, 32):
        feats.append((i, float(i - 20), 60.0, ms("2020-12-%dT%02d:00:00.000Z" % (i, i - 10))))
    ids = np.array([f[0] for f in feats])
    x = np.array([f[1] for f in feats]); y = np.array([f[2] for f in feats]); t = np.array([f[3] for f in feats])
    ks = Z3IndexKeySpace("year")
    b, z, st = oracle.z3_index_key_batch(x, y, t, period=oracle.YEAR)
    assert (st == 0).all()
    for bbox, iv, expected in [
            ((0, 55, 70, 65), during(ms("2020-12-01T00:00:00.000Z"), ms("2020-12-31T23:59:59.999Z")), set(range(32))),
            ((9, 59, 12, 61), during(ms("2020-12-31T00:00:00.000Z"), ms("2020-12-31T23:59:59.999Z")), {31})]:
        v = ks.get_index_values([bbox], [iv])
        # the fake back end (TestGeoMesaDataStore) applies the full ECQL after the range scan
        m = oracle.z3filter_scan(F.serialize_to_bytes(F.Z3Filter.from_values(v)), ks.bin_ranges(v), b, z)
        strict = oracle.strict_scan(x, y, t, bbox, (iv.lower, iv.upper))
        assert set(ids[m & strict].tolist()) == expected
