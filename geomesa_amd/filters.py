"""Row filters pushed down to the key space: Z3Filter / Z2Filter and the strict full filter.

Mirrors geomesa-index-api/src/main/scala/org/locationtech/geomesa/index/filters/:
  * ``Z3Filter``  -- Z3Filter.scala:19-183 (construction from index values :78-110, wire
    formats serializeToBytes/deserializeFromBytes :112-153, serializeToStrings/deserializeFromStrings
    :155-182, inBounds :26-62)
  * ``Z2Filter``  -- Z2Filter.scala:20-61
Byte/string formats are bit-identical to the Scala ones, so a JVM shim hands the serialized
filter straight to ``gm_z3filter_scan``.  Scans run on the GPU (``scan``); there is no host path.
"""
import ctypes
import struct

import numpy as np

from . import _lib
from ._lib import check, ptr

XYKey, TKey, EpochKey, VersionKey = "zxy", "zt", "epoch", "v"
ProjectVersion = "5.3.0-SNAPSHOT-mi355x"
_RS, _TS, _ES = ":", ";", ","


def _i32(v):
    v = int(v)
    if not (-2**31 <= v < 2**31):
        raise ValueError("int32 overflow")
    return v


class Z3Filter:
    """Z3Filter(xy: Array[Array[Int]], t: Array[Array[Array[Int]]], minEpoch: Short, maxEpoch: Short)."""

    def __init__(self, xy, t, min_epoch, max_epoch):
        self.xy = [[_i32(v) for v in b] for b in xy]
        self.t = [None if e is None else [[_i32(v) for v in r] for r in e] for e in t]
        self.minEpoch = int(min_epoch)
        self.maxEpoch = int(max_epoch)

    # Z3Filter.apply(values) (Z3Filter.scala:78-110)
    @classmethod
    def from_values(cls, values):
        sfc = values.sfc
        xy = [[sfc.lon.normalize(a), sfc.lat.normalize(b), sfc.lon.normalize(c), sfc.lat.normalize(d)]
              for (a, b, c, d) in values.spatialBounds]
        whole = [(int(sfc.time.min), int(sfc.time.max))]
        min_e, max_e = 32767, -32768
        eat = []
        for epoch in sorted(values.temporalBounds):
            times = values.temporalBounds[epoch]
            if list(times) == whole:
                continue
            min_e = min(min_e, epoch)
            max_e = max(max_e, epoch)
            eat.append((epoch, [[sfc.time.normalize(t1), sfc.time.normalize(t2)] for (t1, t2) in times]))
        if min_e == 32767 and max_e == -32768:
            t = []
        else:
            t = [None] * (max_e - min_e + 1)
        for (w, times) in eat:
            t[w - min_e] = times
        return cls(xy, t, min_e, max_e)

    def __eq__(self, o):
        return (isinstance(o, Z3Filter) and self.xy == o.xy and self.t == o.t and
                self.minEpoch == o.minEpoch and self.maxEpoch == o.maxEpoch)

    def __repr__(self):
        return ",".join("(%s,%s)" % kv for kv in sorted(serialize_to_strings(self).items()))

    def serialize_to_bytes(self):
        return serialize_to_bytes(self)

    def in_bounds(self, row, offset=0):
        """Single-row Z3Filter.inBounds on row bytes (host convenience for planning/tests)."""
        bins = np.array([struct.unpack_from(">h", row, offset)[0]], np.int16)
        z = np.array([struct.unpack_from(">q", row, offset + 2)[0]], np.int64)
        return bool(scan(self, bins, z)[0].item())


# Z3Filter.serializeToBytes (Z3Filter.scala:112-137)
def serialize_to_bytes(f):
    if isinstance(f, Z2Filter):
        return z2_serialize_to_bytes(f)
    out = [struct.pack(">i", len(f.xy))]
    for b in f.xy:
        out.append(struct.pack(">4i", *b))
    out.append(struct.pack(">i", len(f.t)))
    for bounds in f.t:
        if bounds is None:
            out.append(struct.pack(">i", -1))
        else:
            out.append(struct.pack(">i", len(bounds)))
            for r in bounds:
                out.append(struct.pack(">2i", *r))
    out.append(struct.pack(">hh", f.minEpoch, f.maxEpoch))
    return b"".join(out)


# Z3Filter.deserializeFromBytes (Z3Filter.scala:139-153)
def deserialize_from_bytes(b):
    o = 0
    (nxy,) = struct.unpack_from(">i", b, o); o += 4
    xy = []
    for _ in range(nxy):
        xy.append(list(struct.unpack_from(">4i", b, o))); o += 16
    (nt,) = struct.unpack_from(">i", b, o); o += 4
    t = []
    for _ in range(nt):
        (ln,) = struct.unpack_from(">i", b, o); o += 4
        if ln == -1:
            t.append(None)
        else:
            e = []
            for _ in range(ln):
                e.append(list(struct.unpack_from(">2i", b, o))); o += 8
            t.append(e)
    mn, mx = struct.unpack_from(">hh", b, o)
    return Z3Filter(xy, t, mn, mx)


# Z3Filter.serializeToStrings (Z3Filter.scala:155-170)
def serialize_to_strings(f):
    xy = _TS.join(_RS.join(str(v) for v in b) for b in f.xy)
    t = _ES.join("" if bounds is None else _TS.join(_RS.join(str(v) for v in r) for r in bounds)
                 for bounds in f.t)
    return {XYKey: xy, TKey: t, EpochKey: "%d%s%d" % (f.minEpoch, _RS, f.maxEpoch), VersionKey: ProjectVersion}


def _java_split(s, sep):
    """java.lang.String.split: trailing empty strings removed."""
    parts = s.split(sep)
    while parts and parts[-1] == "":
        parts.pop()
    return parts if parts or s == "" else parts


# Z3Filter.deserializeFromStrings (Z3Filter.scala:172-182)
def deserialize_from_strings(m):
    xy = [[int(v) for v in _java_split(b, _RS)] for b in _java_split(m[XYKey], _TS)] if m[XYKey] else \
        [[int(v) for v in _java_split("", _RS)]]
    t_s = _java_split(m[TKey], _ES)
    if m[TKey] == "":
        t_s = [""]
    t = []
    for bounds in t_s:
        if bounds == "":
            t.append(None)
        else:
            t.append([[int(v) for v in _java_split(r, _RS)] for r in _java_split(bounds, _TS)])
    mn, mx = (int(v) for v in m[EpochKey].split(_RS))
    return Z3Filter(xy, t, mn, mx)


class Z2Filter:
    """Z2Filter(xy) (Z2Filter.scala:20-61)."""

    def __init__(self, xy):
        self.xy = [[_i32(v) for v in b] for b in xy]

    @classmethod
    def from_values(cls, values):
        sfc = values.sfc
        return cls([[sfc.lon.normalize(a), sfc.lat.normalize(b), sfc.lon.normalize(c), sfc.lat.normalize(d)]
                    for (a, b, c, d) in values.spatialBounds])

    def __eq__(self, o):
        return isinstance(o, Z2Filter) and self.xy == o.xy

    def serialize_to_bytes(self):
        return z2_serialize_to_bytes(self)


def z2_serialize_to_bytes(f):
    return struct.pack(">i", len(f.xy)) + b"".join(struct.pack(">4i", *b) for b in f.xy)


def z2_deserialize_from_bytes(b):
    (n,) = struct.unpack_from(">i", b, 0)
    return Z2Filter([list(struct.unpack_from(">4i", b, 4 + 16 * i)) for i in range(n)])


def z2_serialize_to_strings(f):
    return {XYKey: _TS.join(_RS.join(str(v) for v in b) for b in f.xy), VersionKey: ProjectVersion}


def z2_deserialize_from_strings(m):
    return Z2Filter([[int(v) for v in b.split(_RS)] for b in _java_split(m[XYKey], _TS)])


RowOffsetKey = "zo"   # RowFilterIterator.RowOffsetKey (geomesa-accumulo-iterators/.../RowFilterIterator.scala:84-86)


def z3_iterator_options(values, offset, compatibility=None):
    """Z3Iterator.configure's iterator options (geomesa-accumulo-iterators/.../Z3Iterator.scala:30-66).

    compatibility None: the serialized Z3Filter plus the row offset; "1.3": the GeoMesa 1.3 option
    strings -- per bounding box the normalized corners "xmin:ymin:xmax:ymax" joined by ";", per time
    bin (ascending) "bin;t1:t2[;t1:t2...]" joined by ",", through the values' own curve (the legacy
    SemiNormalized dimensions for a Z3IndexKeySpaceV4)."""
    if compatibility is None:
        opts = serialize_to_strings(Z3Filter.from_values(values))
        opts[RowOffsetKey] = str(offset)
        return opts
    if compatibility != "1.3":
        raise NotImplementedError("Unknown compatibility flag: '%s'" % compatibility)
    sfc = values.sfc
    xy = ["%d:%d:%d:%d" % (sfc.lon.normalize(a), sfc.lat.normalize(b), sfc.lon.normalize(c), sfc.lat.normalize(d))
          for (a, b, c, d) in values.spatialBounds]
    ts = []
    for b in sorted(values.temporalBounds):
        ts.append("%d;%s" % (b, _TS.join("%d:%d" % (sfc.time.normalize(t1), sfc.time.normalize(t2))
                                         for (t1, t2) in values.temporalBounds[b])))
    return {XYKey: _TS.join(xy), TKey: _ES.join(ts), RowOffsetKey: str(offset), "zl": "8"}


# ------------------------------------------------------------------------------ GPU scans

def _cols(*pairs):
    from .curve import _dev_col
    return [_dev_col(a, dt) for a, dt in pairs]


def _outputs(n, dev, want_ids, ids_cap):
    import torch
    mask = torch.empty((n + 63) // 64 if n else 1, dtype=torch.int64, device=dev)
    ids = torch.empty(max(ids_cap, 1), dtype=torch.int64, device=dev) if want_ids else None
    return mask, ids


def _mask_to_bool(mask, n):
    import torch
    if n == 0:
        return torch.zeros(0, dtype=torch.bool, device=mask.device)
    bits = torch.arange(64, device=mask.device, dtype=torch.int64)
    m = ((mask.view(-1, 1) >> bits) & 1).view(-1)[:n]
    return m.bool()


def scan(z3filter, bins, z, bin_ranges=(), want_ids=False, ids_cap=None):
    """gm_z3filter_scan: Z3Filter.inBounds over columnar (bin, z) keys restricted to `bin_ranges`.

    Returns (match_bool_tensor, ids_tensor_or_None, n_match)."""
    import torch
    fb = serialize_to_bytes(z3filter) if not isinstance(z3filter, (bytes, bytearray)) else bytes(z3filter)
    bins, z = _cols((bins, torch.int16), (z, torch.int64))
    n = z.numel()
    ctx = _lib.context()
    cap = n if ids_cap is None else ids_cap
    mask, ids = _outputs(n, z.device, want_ids, cap)
    br = np.ascontiguousarray(np.asarray(bin_ranges, np.int16).reshape(-1))
    fbuf = (ctypes.c_uint8 * max(len(fb), 1)).from_buffer_copy(fb if fb else b"\0")
    nm = ctypes.c_int64()
    rc = ctx.lib.gm_z3filter_scan(ctx.handle, fbuf, len(fb),
                                  br.ctypes.data if len(br) else None, len(br) // 2,
                                  ptr(bins), ptr(z), n, ptr(mask), ptr(ids), cap, ctypes.byref(nm))
    if rc != _lib.GM_E_CAPACITY:
        check(rc, "gm_z3filter_scan")
    m = _mask_to_bool(mask, n)
    return m, (ids[:min(nm.value, cap)] if want_ids else None), nm.value


def z2_scan(z2filter, z, want_ids=False, ids_cap=None):
    import torch
    fb = z2_serialize_to_bytes(z2filter) if not isinstance(z2filter, (bytes, bytearray)) else bytes(z2filter)
    (z,) = _cols((z, torch.int64))
    n = z.numel()
    ctx = _lib.context()
    cap = n if ids_cap is None else ids_cap
    mask, ids = _outputs(n, z.device, want_ids, cap)
    fbuf = (ctypes.c_uint8 * len(fb)).from_buffer_copy(fb)
    nm = ctypes.c_int64()
    rc = ctx.lib.gm_z2filter_scan(ctx.handle, fbuf, len(fb), ptr(z), n, ptr(mask), ptr(ids), cap, ctypes.byref(nm))
    if rc != _lib.GM_E_CAPACITY:
        check(rc, "gm_z2filter_scan")
    return _mask_to_bool(mask, n), (ids[:min(nm.value, cap)] if want_ids else None), nm.value


def scan_rows(row_filter, rows, row_off, key_offset=0, want_ids=False, ids_cap=None):
    """RowFilter.inBounds(row, key_offset) for every row of a batch of row-key bytes (the loop of
    RowFilterIterator.findTop, RowFilterIterator.scala:52-66): gm_z3filter_scan_rows for a Z3Filter
    (or its serialized bytes with kind "z3"), gm_z2filter_scan_rows for a Z2Filter.  rows = all row
    bytes back to back (uint8), row_off = n + 1 int64 offsets.  Returns (mask, ids, n_match, n_short)."""
    import torch
    if isinstance(row_filter, Z2Filter):
        fb, fn = z2_serialize_to_bytes(row_filter), "gm_z2filter_scan_rows"
    else:
        fb = serialize_to_bytes(row_filter) if isinstance(row_filter, Z3Filter) else bytes(row_filter)
        fn = "gm_z3filter_scan_rows"
    ctx = _lib.context()
    dev = torch.device("cuda", ctx.device)
    rows = rows.to(dev) if isinstance(rows, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(np.frombuffer(bytes(rows), np.uint8).copy() if isinstance(rows, (bytes, bytearray))
                             else np.asarray(rows, np.uint8))).to(dev)
    if rows.numel() == 0:
        rows = torch.zeros(4, dtype=torch.uint8, device=dev)
    (row_off,) = _cols((row_off, torch.int64))
    n = row_off.numel() - 1
    cap = n if ids_cap is None else ids_cap
    mask, ids = _outputs(n, dev, want_ids, cap)
    fbuf = (ctypes.c_uint8 * len(fb)).from_buffer_copy(fb)
    nm, ns = ctypes.c_int64(), ctypes.c_int64()
    rc = getattr(ctx.lib, fn)(ctx.handle, fbuf, len(fb), ptr(rows), ptr(row_off), int(key_offset), n, ptr(mask),
                              ptr(ids), cap, ctypes.byref(nm), ctypes.byref(ns))
    if rc != _lib.GM_E_CAPACITY:
        check(rc, fn)
    return _mask_to_bool(mask, n), (ids[:min(nm.value, cap)] if want_ids else None), nm.value, ns.value


def strict_scan(x, y, t_ms, bbox, during=None, want_ids=False, ids_cap=None):
    """Full-filter evaluation: BBOX (inclusive, GeometryProcessing.scala:129) AND FastDuring
    (exclusive, FastTemporalOperator.scala:123-126) on raw columns."""
    import torch
    x, y = _cols((x, torch.float64), (y, torch.float64))
    n = x.numel()
    t = _cols((t_ms, torch.int64))[0] if during is not None else None
    ctx = _lib.context()
    cap = n if ids_cap is None else ids_cap
    mask, ids = _outputs(n, x.device, want_ids, cap)
    bb = (ctypes.c_double * 4)(*[float(v) for v in bbox])
    lo, hi = during if during is not None else (0, 0)
    nm = ctypes.c_int64()
    rc = ctx.lib.gm_strict_scan(ctx.handle, ptr(x), ptr(y), ptr(t), n, bb, int(during is not None), int(lo), int(hi),
                                ptr(mask), ptr(ids), cap, ctypes.byref(nm))
    if rc != _lib.GM_E_CAPACITY:
        check(rc, "gm_strict_scan")
    return _mask_to_bool(mask, n), (ids[:min(nm.value, cap)] if want_ids else None), nm.value


SPATIAL_OPS = {None: _lib.GM_SPATIAL_NONE, "intersects": _lib.GM_SPATIAL_INTERSECTS,
               "contains": _lib.GM_SPATIAL_CONTAINS, "within": _lib.GM_SPATIAL_CONTAINS}


def query_scan(x, y, t_ms=None, bbox=None, during=None, geoms=None, op="intersects", want_ids=False, ids_cap=None):
    """The full filter of a point query in one pass (gm_query_scan): BBOX (inclusive) AND during
    (exclusive ms) AND, over the polygons of `geoms` (a join.PolygonIndex, or a join.PolygonSet that
    is indexed here), OR of INTERSECTS(geom, P) (op "intersects") or CONTAINS(P, geom) /
    WITHIN(geom, P) (op "contains" / "within").  Absent terms (None) are left out.
    Returns (mask, ids, n_match) like strict_scan."""
    import torch
    from .join import PolygonIndex, PolygonSet
    x, y = _cols((x, torch.float64), (y, torch.float64))
    n = x.numel()
    t = _cols((t_ms, torch.int64))[0] if during is not None else None
    if geoms is None:
        op = None
    elif isinstance(geoms, PolygonSet):
        geoms = PolygonIndex(geoms, cells_per_poly=65536)
    if op not in SPATIAL_OPS:
        raise ValueError("spatial op must be one of %s" % sorted(k for k in SPATIAL_OPS if k))
    ctx = _lib.context()
    cap = n if ids_cap is None else ids_cap
    mask, ids = _outputs(n, x.device, want_ids, cap)
    bb = (ctypes.c_double * 4)(*[float(v) for v in bbox]) if bbox is not None else None
    lo, hi = during if during is not None else (0, 0)
    nm = ctypes.c_int64()
    rc = ctx.lib.gm_query_scan(ctx.handle, ptr(x), ptr(y), ptr(t), n, bb, int(during is not None), int(lo), int(hi),
                               geoms._h if geoms is not None else None, SPATIAL_OPS[op], ptr(mask), ptr(ids), cap,
                               ctypes.byref(nm))
    if rc != _lib.GM_E_CAPACITY:
        check(rc, "gm_query_scan")
    return _mask_to_bool(mask, n), (ids[:min(nm.value, cap)] if want_ids else None), nm.value
