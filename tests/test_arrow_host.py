"""Arrow columnar input, host side (no GPU): the buffers a gm_geom_column points at decode back to the
same geometries pyarrow sees (slices, nulls, every nesting depth, Float4), and the oracle's JTS
envelope rules on hand-checked cases (JTS 1.20 Geometry.getEnvelopeInternal -- parity unpinned by a
reference fixture: the reference holds no Arrow golden files for envelopes; the rules are restated)."""
import numpy as np
import pyarrow as pa
import pytest

from geomesa_amd.arrow import arrow_buffers

PT = pa.list_(pa.float64(), 2)
PT4 = pa.list_(pa.float32(), 2)
TYPES = {
    "point": PT, "linestring": pa.list_(PT), "multipoint": pa.list_(PT), "polygon": pa.list_(pa.list_(PT)),
    "multilinestring": pa.list_(pa.list_(PT)), "multipolygon": pa.list_(pa.list_(pa.list_(PT))),
}
DEPTH = {"point": 0, "linestring": 1, "multipoint": 1, "polygon": 2, "multilinestring": 2, "multipolygon": 3}


def decode(arr, kind):
    """Walk the extracted buffers exactly as the device kernels do."""
    coords, bits, valid, voff, offs = arrow_buffers(arr, kind)
    out = []

    def tuples(a, b):
        return [[float(coords[2 * j]), float(coords[2 * j + 1])] for j in range(a, b)]

    def nest(level, a, b):
        if level == len(offs):
            return tuples(a, b)
        o = offs[level]
        return [nest(level + 1, o[k], o[k + 1]) for k in range(a, b)]
    for i in range(len(arr)):
        if valid is not None and not (valid[(voff + i) >> 3] >> ((voff + i) & 7)) & 1:
            out.append(None)
        elif kind == "point":
            out.append(tuples(i, i + 1)[0])
        else:
            o = offs[0]
            out.append(nest(1, o[i], o[i + 1]) if len(offs) > 1 else tuples(o[i], o[i + 1]))
    return out


def rand_geom(rng, depth):
    if depth == 0:
        return [float(rng.uniform(-90, 90)), float(rng.uniform(-180, 180))]
    return [rand_geom(rng, depth - 1) for _ in range(int(rng.integers(0, 4)))]


@pytest.mark.parametrize("kind", sorted(TYPES))
def test_buffers_decode_with_slices_and_nulls(kind):
    rng = np.random.default_rng(7)
    vals = [None if rng.uniform() < 0.2 else rand_geom(rng, DEPTH[kind]) for _ in range(57)]
    arr = pa.array(vals, TYPES[kind])
    for a, b in [(0, 57), (3, 50), (13, 14), (20, 20)]:
        s = arr.slice(a, b - a)
        assert decode(s, kind) == s.to_pylist()


def test_float4_points_and_child_offsets():
    vals = [[1.5, -2.25], None, [3.0, 4.0], [5.0, 6.5]]
    arr = pa.array(vals, PT4).slice(1)
    coords, bits, valid, voff, offs = arrow_buffers(arr, "point")
    assert bits == 32 and coords.dtype == np.float32 and voff == 1
    assert decode(arr, "point") == arr.to_pylist()


def test_rejects_non_geometry_layouts():
    from geomesa_amd.curve import IllegalArgumentException
    with pytest.raises(IllegalArgumentException):
        arrow_buffers(pa.array([[1.0, 2.0, 3.0]], pa.list_(pa.float64(), 3)), "point")
    with pytest.raises(IllegalArgumentException):
        arrow_buffers(pa.array([[1, 2]], pa.list_(pa.int32(), 2)), "point")
    with pytest.raises(IllegalArgumentException):
        arrow_buffers(pa.array([[1.0, 2.0]], PT), "polygon")


def test_oracle_envelopes(oracle):
    O = oracle
    # tuples are [y, x]
    shell = [[0.0, 0.0], [0.0, 10.0], [5.0, 10.0], [5.0, 0.0], [0.0, 0.0]]
    hole_outside = [[50.0, 50.0], [50.0, 60.0], [60.0, 60.0], [50.0, 50.0]]
    arr = pa.array([[shell, hole_outside], [], None], TYPES["polygon"])
    rows = O.arrow_rows(arr, "polygon")
    assert O.jts_envelope(rows[0], "polygon") == (0.0, 0.0, 10.0, 5.0)   # shell only
    assert O.jts_envelope(rows[1], "polygon") == (0.0, 0.0, -1.0, -1.0)  # empty: null envelope
    mp = pa.array([[[shell], [], [[[-3.0, 20.0], [-1.0, 21.0], [-3.0, 20.0]]]]], TYPES["multipolygon"])
    assert O.jts_envelope(O.arrow_rows(mp, "multipolygon")[0], "multipolygon") == (0.0, -3.0, 21.0, 5.0)
    # flipAxisOrder: tuples [x, y]
    assert O.arrow_rows(pa.array([[1.0, 2.0]], PT), "point", flip_axis=True) == [(1.0, 2.0)]
    # the null envelope fails XZ2's ordering require; a null slot is the null-geometry error
    z, st = O.arrow_xz2_keys(arr, "polygon")
    assert st.tolist() == [O.OK, O.UNORDERED, O.NULL_GEOM]
    assert z[0] == O.xz2_index(0.0, 0.0, 10.0, 5.0)[1]


def test_oracle_arrow_keys_match_columns(oracle):
    O = oracle
    rng = np.random.default_rng(3)
    n = 200
    x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n)
    t = rng.integers(1577836800000, 1609459200000, n)
    arr = pa.array([[float(b), float(a)] for a, b in zip(x, y)], PT)
    b, z, st = O.arrow_z3_keys(arr, pa.array(t, pa.timestamp("ms")))
    ob, oz, ost = O.z3_index_key_batch(x, y, t)
    assert np.array_equal(b, ob) and np.array_equal(z, oz) and np.array_equal(st, ost)
    # a null date is time 0 (Z3IndexKeySpace.scala:71-72)
    b, z, st = O.arrow_z3_keys(arr, pa.array([None] * n, pa.timestamp("ms")))
    ob, oz, _ = O.z3_index_key_batch(x, y, np.zeros(n, np.int64))
    assert np.array_equal(b, ob) and np.array_equal(z, oz)
