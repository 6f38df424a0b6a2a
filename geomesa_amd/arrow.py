"""Arrow columnar input: GeoMesa's Arrow geometry vectors as zero-copy device input.

GeoMesa's JVM side already carries feature batches as Arrow vectors (geomesa-arrow-jts); this module
hands such vectors to the C-ABI without building per-feature JTS objects:

  * PointVector / PointFloatVector  -- FixedSizeList(2) of Float8 / Float4, tuples [y, x] unless
    flipAxisOrder (geomesa-arrow-jts/.../impl/AbstractPointVector.java:52-79);
  * LineStringVector, MultiPointVector -- List<FixedSizeList(2)> (AbstractLineStringVector.java);
  * PolygonVector, MultiLineStringVector -- List<List<FixedSizeList(2)>>, rings shell first
    (AbstractPolygonVector.java:56-84);
  * MultiPolygonVector -- List<List<List<FixedSizeList(2)>>> (AbstractMultiPolygonVector.java:61-95).

A pyarrow Array of one of those shapes becomes a GeometryColumn: its buffers are copied to HBM once
(the stand-in for the JVM handing over off-heap Arrow buffers that already live on the device) and
passed by pointer, with the array offsets and validity bitmaps as they are.  The entry points mirror
the key spaces' toIndexKey over a batch:
  Z3IndexKeySpace.toIndexKey  (idx/index/z3/Z3IndexKeySpace.scala:63-95)
  Z2IndexKeySpace.toIndexKey  (idx/index/z2/Z2IndexKeySpace.scala:48-75)
  XZ2IndexKeySpace.toIndexKey (idx/index/z2/XZ2IndexKeySpace.scala:48-76)
  XZ3IndexKeySpace.toIndexKey (idx/index/z3/XZ3IndexKeySpace.scala:60-95)
and the st_contains join over an Arrow point column against an Arrow polygon column.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, ptr
from .curve import IllegalArgumentException, TimePeriod, _raise_first, _summary

KINDS = {"point": 0, "linestring": 1, "polygon": 2, "multipoint": 3, "multilinestring": 4, "multipolygon": 5}
LEVELS = {"point": 0, "linestring": 1, "multipoint": 1, "polygon": 2, "multilinestring": 2, "multipolygon": 3}


class GeomColumnC(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("ordinal_bits", ctypes.c_int32), ("flip_axis", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("coords", ctypes.c_void_p), ("validity", ctypes.c_void_p),
                ("validity_offset", ctypes.c_int64), ("offsets", ctypes.c_void_p * 3)]


class TimeColumnC(ctypes.Structure):
    _fields_ = [("millis", ctypes.c_void_p), ("validity", ctypes.c_void_p), ("validity_offset", ctypes.c_int64)]


def _validity(arr):
    """(bitmap bytes or None, bit offset) of an Arrow array's top-level validity."""
    if arr.null_count == 0:
        return None, 0
    buf = arr.buffers()[0]
    return np.frombuffer(buf, np.uint8), arr.offset


def _offsets(arr):
    """Int32 List offsets of `arr` with its array offset applied (n + 1 entries)."""
    import pyarrow as pa
    if not pa.types.is_list(arr.type):
        raise IllegalArgumentException("expected an Arrow List level, got %s" % arr.type)
    return np.asarray(arr.offsets.to_numpy(zero_copy_only=False), np.int32)


def _tuples(fsl):
    """Ordinate buffer of a FixedSizeList(2) array, tuple j of `fsl` at [2j], [2j + 1]."""
    import pyarrow as pa
    if not (pa.types.is_fixed_size_list(fsl.type) and fsl.type.list_size == 2):
        raise IllegalArgumentException("expected FixedSizeList(2) tuples, got %s" % fsl.type)
    vals = fsl.values                       # the child, ignoring fsl's own offset
    vt = vals.type
    if pa.types.is_float64(vt):
        dt, bits = np.float64, 64
    elif pa.types.is_float32(vt):
        dt, bits = np.float32, 32
    else:
        raise IllegalArgumentException("ordinates must be Float8 or Float4, got %s" % vt)
    flat = np.frombuffer(vals.buffers()[1], dt)
    start = vals.offset + 2 * fsl.offset
    return flat[start:start + 2 * len(fsl)], bits


def arrow_buffers(arr, kind):
    """The buffers a gm_geom_column points at, host side: (ordinates, ordinal bits, validity bitmap or
    None, validity bit offset, [List offsets, outermost first])."""
    kind = kind.lower()
    if kind not in KINDS:
        raise IllegalArgumentException("unknown geometry kind %r" % kind)
    valid, voff = _validity(arr)
    offs = []
    level = arr
    for _ in range(LEVELS[kind]):
        offs.append(_offsets(level))
        level = level.values
    coords, bits = _tuples(level)
    return coords, bits, valid, voff, offs


class GeometryColumn:
    """A geomesa-arrow-jts geometry vector (as a pyarrow Array) resident on the device."""

    def __init__(self, arr, kind, flip_axis=False, device=None):
        import torch
        import pyarrow as pa
        if isinstance(arr, pa.ChunkedArray):
            arr = arr.combine_chunks()
        kind = kind.lower()
        self.kind, self.n, self.flip_axis = kind, len(arr), bool(flip_axis)
        coords, self.ordinal_bits, valid, voff, offs = arrow_buffers(arr, kind)
        ctx = _lib.context(device)
        dev = torch.device("cuda", ctx.device)

        def up(a):
            return torch.from_numpy(np.array(a)).to(dev) if a is not None else None
        # a zero-length buffer still gets a valid pointer
        self._coords = up(coords if len(coords) else np.zeros(2, coords.dtype))
        self._valid = up(valid)
        self._offs = [up(o) for o in offs]
        self._host = (coords, valid, offs)   # keeps host views alive for the host-side index build
        self._c = GeomColumnC(KINDS[kind], self.ordinal_bits, int(self.flip_axis), 0, self._coords.data_ptr(),
                              self._valid.data_ptr() if self._valid is not None else None, voff,
                              (ctypes.c_void_p * 3)(*([o.data_ptr() for o in self._offs] +
                                                      [None] * (3 - len(self._offs)))))
        self._voff = voff

    def c_struct(self):
        return self._c

    def host_struct(self):
        """The same column with host pointers (gm_pip_index_create_arrow reads host memory)."""
        coords, valid, offs = self._host
        if not len(coords):
            coords = np.zeros(2, coords.dtype)
        self._host_keep = (np.ascontiguousarray(coords), None if valid is None else np.ascontiguousarray(valid),
                           [np.ascontiguousarray(o) for o in offs])
        c, v, o = self._host_keep
        return GeomColumnC(KINDS[self.kind], self.ordinal_bits, int(self.flip_axis), 0, c.ctypes.data,
                           v.ctypes.data if v is not None else None, self._voff,
                           (ctypes.c_void_p * 3)(*([a.ctypes.data for a in o] + [None] * (3 - len(o)))))


class TimeColumn:
    """An Arrow date column (Timestamp(ms) / Date64 / Int64 epoch millis) resident on the device."""

    def __init__(self, arr, device=None):
        import torch
        import pyarrow as pa
        if isinstance(arr, pa.ChunkedArray):
            arr = arr.combine_chunks()
        t = arr.type
        if pa.types.is_timestamp(t):
            if t.unit != "ms":
                raise IllegalArgumentException("timestamps must be in milliseconds (Arrow TimeStampMilli)")
        elif not (pa.types.is_date64(t) or pa.types.is_int64(t)):
            raise IllegalArgumentException("dates must be Timestamp(ms), Date64 or Int64, got %s" % t)
        self.n = len(arr)
        ctx = _lib.context(device)
        dev = torch.device("cuda", ctx.device)
        ms = np.frombuffer(arr.buffers()[1], np.int64)[arr.offset:arr.offset + len(arr)]
        valid, voff = _validity(arr)
        self._ms = torch.from_numpy(np.array(ms) if len(ms) else np.zeros(1, np.int64)).to(dev)
        self._valid = torch.from_numpy(valid.copy()).to(dev) if valid is not None else None
        self._c = TimeColumnC(self._ms.data_ptr(), self._valid.data_ptr() if self._valid is not None else None,
                              voff)

    def c_struct(self):
        return self._c


def _as_geom(col, kind, flip_axis):
    return col if isinstance(col, GeometryColumn) else GeometryColumn(col, kind, flip_axis)


def _as_time(col):
    if col is None or isinstance(col, TimeColumn):
        return col
    return TimeColumn(col)


def _finish(st, what, status_t, outs):
    if status_t is not None:
        return outs + (status_t,)
    if st.n_errors > 0 and st.first_code == _lib.GM_ST_NULL_GEOM:
        raise IllegalArgumentException("%s: Null geometry in feature (element %d)" % (what, st.first_index))
    _raise_first(st, what)
    return outs if len(outs) > 1 else outs[0]


def z3_index_keys(points, dtg=None, period=TimePeriod.Week, lenient=False, status=False, flip_axis=False):
    """Z3IndexKeySpace.toIndexKey's (bin, z) over an Arrow point column and date column.

    A null date (column or slot) is time 0 (Z3IndexKeySpace.scala:71-72); a null point is the
    "Null geometry in feature" error (:66-68), status GM_ST_NULL_GEOM."""
    import torch
    g = _as_geom(points, "point", flip_axis)
    t = _as_time(dtg)
    if g.kind != "point":
        raise IllegalArgumentException("Z3 keys index point geometries")
    n = g.n
    ctx = _lib.context()
    dev = g._coords.device
    b = torch.empty(n, dtype=torch.int16, device=dev)
    z = torch.empty(n, dtype=torch.int64, device=dev)
    s = torch.empty(n, dtype=torch.uint8, device=dev) if status else None
    st = _summary()
    check(ctx.lib.gm_z3_index_key_arrow(ctx.handle, ctypes.byref(g.c_struct()),
                                        ctypes.byref(t.c_struct()) if t is not None else None, n,
                                        TimePeriod.of(period), int(bool(lenient)), ptr(b), ptr(z), ptr(s),
                                        ctypes.byref(st)), "gm_z3_index_key_arrow")
    return _finish(st, "Z3IndexKeySpace.toIndexKey", s, (b, z))


def z2_index_keys(points, lenient=False, status=False, flip_axis=False):
    """Z2IndexKeySpace.toIndexKey's z over an Arrow point column (Z2IndexKeySpace.scala:48-75)."""
    import torch
    g = _as_geom(points, "point", flip_axis)
    if g.kind != "point":
        raise IllegalArgumentException("Z2 keys index point geometries")
    n = g.n
    ctx = _lib.context()
    z = torch.empty(n, dtype=torch.int64, device=g._coords.device)
    s = torch.empty(n, dtype=torch.uint8, device=g._coords.device) if status else None
    st = _summary()
    check(ctx.lib.gm_z2_index_key_arrow(ctx.handle, ctypes.byref(g.c_struct()), n, int(bool(lenient)), ptr(z),
                                        ptr(s), ctypes.byref(st)), "gm_z2_index_key_arrow")
    return _finish(st, "Z2IndexKeySpace.toIndexKey", s, (z,))


def xz2_index_keys(geoms, kind="polygon", g=12, lenient=False, status=False, flip_axis=False):
    """XZ2IndexKeySpace.toIndexKey over an Arrow geometry column: XZ2SFC(g).index of each JTS
    envelope (XZ2IndexKeySpace.scala:48-76).  An empty geometry's null envelope fails the XZ
    ordering require (GM_ST_UNORDERED)."""
    import torch
    col = _as_geom(geoms, kind, flip_axis)
    n = col.n
    ctx = _lib.context()
    xz = torch.empty(n, dtype=torch.int64, device=col._coords.device)
    s = torch.empty(n, dtype=torch.uint8, device=col._coords.device) if status else None
    st = _summary()
    check(ctx.lib.gm_xz2_index_key_arrow(ctx.handle, ctypes.byref(col.c_struct()), n, int(g), int(bool(lenient)),
                                         ptr(xz), ptr(s), ctypes.byref(st)), "gm_xz2_index_key_arrow")
    return _finish(st, "XZ2IndexKeySpace.toIndexKey", s, (xz,))


def xz3_index_keys(geoms, dtg=None, kind="polygon", g=12, period=TimePeriod.Week, lenient=False, status=False,
                   flip_axis=False):
    """XZ3IndexKeySpace.toIndexKey's (bin, xz) over an Arrow geometry + date column
    (XZ3IndexKeySpace.scala:60-95)."""
    import torch
    col = _as_geom(geoms, kind, flip_axis)
    t = _as_time(dtg)
    n = col.n
    ctx = _lib.context()
    dev = col._coords.device
    b = torch.empty(n, dtype=torch.int16, device=dev)
    xz = torch.empty(n, dtype=torch.int64, device=dev)
    s = torch.empty(n, dtype=torch.uint8, device=dev) if status else None
    st = _summary()
    check(ctx.lib.gm_xz3_index_key_arrow(ctx.handle, ctypes.byref(col.c_struct()),
                                         ctypes.byref(t.c_struct()) if t is not None else None, n, int(g),
                                         TimePeriod.of(period), int(bool(lenient)), ptr(b), ptr(xz), ptr(s),
                                         ctypes.byref(st)), "gm_xz3_index_key_arrow")
    return _finish(st, "XZ3IndexKeySpace.toIndexKey", s, (b, xz))


def points_to_columns(points, flip_axis=False):
    """(x, y) float64 device columns of an Arrow point column; null points are NaN."""
    import torch
    g = _as_geom(points, "point", flip_axis)
    n = g.n
    ctx = _lib.context()
    xy = torch.empty(2 * max(n, 1), dtype=torch.float64, device=g._coords.device)
    x, y = xy[:n], xy[max(n, 1):max(n, 1) + n]
    check(ctx.lib.gm_arrow_points_to_columns(ctx.handle, ctypes.byref(g.c_struct()), n, ptr(x), ptr(y)),
          "gm_arrow_points_to_columns")
    return x, y


class ArrowPolygonIndex:
    """The join index built from an Arrow Polygon / MultiPolygon column (null slots never match)."""

    def __init__(self, polys, kind="polygon", flip_axis=False, cells_per_poly=0):
        from .join import PolygonIndex
        col = _as_geom(polys, kind, flip_axis)
        if col.kind not in ("polygon", "multipolygon"):
            raise IllegalArgumentException("the join's polygon side must be Polygon or MultiPolygon")
        self.ctx = _lib.context()
        hs = col.host_struct()
        h = ctypes.c_void_p()
        check(self.ctx.lib.gm_pip_index_create_arrow(self.ctx.handle, ctypes.byref(hs), col.n, int(cells_per_poly),
                                                     ctypes.byref(h)), "gm_pip_index_create_arrow")
        self._col = col
        # reuse PolygonIndex's lifetime handling and join() on x / y columns
        self.index = PolygonIndex.__new__(PolygonIndex)
        self.index.polyset, self.index.ctx, self.index._h = None, self.ctx, h

    def join(self, points, id_base=0, cap=None, count_only=False, mode="auto", flip_axis=False,
             predicate="st_contains"):
        """(pt_ids, poly_ids) with predicate(poly, point) over an Arrow point column."""
        import torch
        g = _as_geom(points, "point", flip_axis)
        n = g.n
        m = self.index.MODES[mode]
        pr = self.index.PREDICATES[predicate]
        npairs = ctypes.c_int64()
        lib, hctx, hix = self.ctx.lib, self.ctx.handle, self.index._h
        if count_only:
            check(lib.gm_pip_join_arrow(hctx, hix, ctypes.byref(g.c_struct()), n, id_base, None, None, 0,
                                        ctypes.byref(npairs), m, pr), "gm_pip_join_arrow")
            return npairs.value
        if cap is None:
            cap = max(1024, n + n // 4)
        dev = g._coords.device
        while True:
            pt = torch.empty(cap, dtype=torch.int64, device=dev)
            pl = torch.empty(cap, dtype=torch.int32, device=dev)
            rc = lib.gm_pip_join_arrow(hctx, hix, ctypes.byref(g.c_struct()), n, id_base, ptr(pt), ptr(pl), cap,
                                       ctypes.byref(npairs), m, pr)
            if rc == _lib.GM_E_CAPACITY:
                cap = npairs.value
                continue
            check(rc, "gm_pip_join_arrow")
            k = npairs.value
            return pt[:k], pl[:k]
