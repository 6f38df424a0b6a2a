"""Batched range decomposition on the GPU (gm_z3_ranges / gm_z2_ranges / gm_xz2_ranges / gm_xz3_ranges).

One ZN.zranges (geomesa-z3/.../zorder/sfcurve/ZN.scala:110-242) or XZ ranges walk
(curve/XZ2SFC.scala:146-252, XZ3SFC.scala:156-262) per query, all queries in one launch.
Results are lists of IndexRange identical to the Scala output (same truncation, sort and merge).
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check
from .curve import IllegalArgumentException, IndexRange

_QS_MSG = {1: "Value(s) out of bounds", 3: "Bounds must be ordered", 4: "range workspace capacity exceeded",
           5: "too many bounds in one query (max 256)"}


RANGE_DTYPE = np.dtype([("lower", "<i8"), ("upper", "<i8"), ("contained", "<i4"), ("reserved", "<i4")])


class RangeList:
    """Ranges of one query: a sequence of IndexRange backed by the numpy result of the batch."""

    def __init__(self, arr):
        self.arr = arr

    def __len__(self):
        return len(self.arr)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        r = self.arr[i]
        return IndexRange(int(r["lower"]), int(r["upper"]), bool(r["contained"]))

    def __iter__(self):
        lo, hi, c = self.arr["lower"].tolist(), self.arr["upper"].tolist(), self.arr["contained"].tolist()
        return (IndexRange(a, b, bool(k)) for a, b, k in zip(lo, hi, c))

    def __eq__(self, o):
        return list(self) == list(o)

    def __repr__(self):
        return repr(list(self))


_pinned = [None]


def _pinned_out(cap):
    """A reusable page-locked output buffer: the library copies results straight into pinned host
    memory (pageable destinations go through its staging buffer, ~8 GB/s)."""
    buf = _pinned[0]
    if buf is None or buf.shape[0] < cap:
        import torch
        t = torch.empty(int(cap * 1.25) * RANGE_DTYPE.itemsize, dtype=torch.uint8, pin_memory=True)
        _pinned[0] = buf = t.numpy().view(RANGE_DTYPE)
        _pinned.append(t)   # keep the tensor (owner of the memory) alive
        del _pinned[1:-1]
    return buf[:cap]


def call_raw(fn, args, nq, cap, pinned=False):
    """Runs one batched ranges entry point; returns (offsets[nq+1], ranges structured array, status).
    pinned=True writes into a reused page-locked buffer (valid until the next pinned call)."""
    cap = max(int(cap), 1024)
    while True:
        out_off = np.zeros(nq + 1, np.int64)
        out = _pinned_out(cap) if pinned else np.empty(cap, RANGE_DTYPE)   # written up to out_off[-1]
        needed = ctypes.c_int64()
        qst = np.zeros(max(nq, 1), np.int32)
        rc = fn(*args, out_off.ctypes.data, out.ctypes.data, cap, ctypes.byref(needed), qst.ctypes.data)
        if rc == _lib.GM_E_CAPACITY:
            cap = needed.value + 1024
            continue
        check(rc, fn.__name__)
        return out_off, out, qst


def _run(fn, args, nq, cap):
    out_off, out, qst = call_raw(fn, args, nq, cap)
    res = []
    for q in range(nq):
        if qst[q] != 0:
            raise IllegalArgumentException("query %d: %s" % (q, _QS_MSG.get(int(qst[q]), "error %d" % qst[q])))
        res.append(RangeList(out[int(out_off[q]):int(out_off[q + 1])]))
    return res


def _mr(max_ranges):
    return 0 if max_ranges is None else int(max_ranges)


def z3_ranges(sfc, queries, precision=64, max_ranges=None, max_recurse=None):
    """queries: [(xy boxes [(xmin, ymin, xmax, ymax)], t intervals [(tmin, tmax)])]."""
    return _run(*prepare_z3(sfc, queries, precision, max_ranges, max_recurse))


def prepare_z3(sfc, queries, precision=64, max_ranges=None, max_recurse=None):
    """(entry point, argument tuple, n_queries, capacity) for gm_z3_ranges (host arrays kept alive)."""
    ctx = _lib.context()
    nq = len(queries)
    box_off, time_off, xy, tt = [0], [0], [], []
    for (bxs, ts) in queries:
        for b in bxs:
            xy.extend(float(v) for v in b)
        for t in ts:
            tt.extend(int(v) for v in t)
        box_off.append(len(xy) // 4)
        time_off.append(len(tt) // 2)
    bo = np.asarray(box_off, np.int32); to = np.asarray(time_off, np.int32)
    xya = np.asarray(xy if xy else [0.0], np.float64); ta = np.asarray(tt if tt else [0], np.int64)
    cap = nq * (max_ranges + 16 if max_ranges else 4096)
    args = (ctx.handle, nq, bo.ctypes.data, xya.ctypes.data, to.ctypes.data, ta.ctypes.data, sfc.period,
            sfc.precision, int(precision), _mr(max_ranges), -1 if max_recurse is None else int(max_recurse))
    _keep.append((bo, to, xya, ta))
    del _keep[:-8]
    return ctx.lib.gm_z3_ranges, args, nq, cap


_keep = []


def z2_ranges(sfc, queries, precision=64, max_ranges=None, max_recurse=None):
    ctx = _lib.context()
    nq = len(queries)
    box_off, xy = [0], []
    for bxs in queries:
        for b in bxs:
            xy.extend(float(v) for v in b)
        box_off.append(len(xy) // 4)
    bo = np.asarray(box_off, np.int32)
    xya = np.asarray(xy if xy else [0.0], np.float64)
    cap = nq * (max_ranges + 16 if max_ranges else 4096)
    args = (ctx.handle, nq, bo.ctypes.data, xya.ctypes.data, sfc.precision, int(precision), _mr(max_ranges),
            -1 if max_recurse is None else int(max_recurse))
    return _run(ctx.lib.gm_z2_ranges, args, nq, cap)


def zranges(dims, queries, precision=64, max_ranges=None, max_recurse=None):
    """ZN.zranges(Array[ZRange], precision, maxRanges, maxRecurse) (zorder/sfcurve/ZN.scala:110-113)
    as Z3.zranges (dims 3) / Z2.zranges (dims 2), one call per query of raw (min, max) z bounds.
    max_recurse None = the Scala default Some(ZN.DefaultRecurse) = 7."""
    ctx = _lib.context()
    nq = len(queries)
    off, zb = [0], []
    for bounds in queries:
        for (lo, hi) in bounds:
            zb.extend((int(lo), int(hi)))
        off.append(len(zb) // 2)
    bo = np.asarray(off, np.int32)
    za = np.asarray(zb if zb else [0], np.int64)
    cap = nq * (max_ranges + 16 if max_ranges else 4096)
    args = (ctx.handle, int(dims), nq, bo.ctypes.data, za.ctypes.data, int(precision), _mr(max_ranges),
            -1 if max_recurse is None else int(max_recurse))
    return _run(ctx.lib.gm_zranges, args, nq, cap)


def _windows(queries, dims):
    off, w = [0], []
    for wins in queries:
        for q in wins:
            q = [float(v) for v in q]
            if len(q) != 2 * dims:
                raise ValueError("window needs %d values" % (2 * dims))
            w.extend(q)
        off.append(len(w) // (2 * dims))
    return np.asarray(off, np.int32), np.asarray(w if w else [0.0], np.float64)


def xz2_ranges(sfc, queries, max_ranges=None):
    """queries: [[(xmin, ymin, xmax, ymax), ...]] -- each query is a list of OR'd windows."""
    ctx = _lib.context()
    nq = len(queries)
    off, w = _windows(queries, 2)
    cap = nq * (4 * max_ranges + 64 if max_ranges else 4096)
    args = (ctx.handle, nq, off.ctypes.data, w.ctypes.data, sfc.g, _mr(max_ranges))
    return _run(ctx.lib.gm_xz2_ranges, args, nq, cap)


def xz3_ranges(sfc, queries, max_ranges=None):
    """queries: [[(xmin, ymin, zmin, xmax, ymax, zmax), ...]]."""
    ctx = _lib.context()
    nq = len(queries)
    off, w = _windows(queries, 3)
    cap = nq * (8 * max_ranges + 64 if max_ranges else 4096)
    args = (ctx.handle, nq, off.ctypes.data, w.ctypes.data, sfc.g, sfc.period, _mr(max_ranges))
    return _run(ctx.lib.gm_xz3_ranges, args, nq, cap)
