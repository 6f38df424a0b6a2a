"""ctypes wrapper around the C restatement (oracle/gm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg -- never by the geomesa_amd product package.
"""
import ctypes
import os
import subprocess

import numpy as np

# gmo_range {int64 lower, upper; int32 contained, pad}: the layout of the library's gm_range
RANGE_DTYPE = np.dtype([("lower", "<i8"), ("upper", "<i8"), ("contained", "<i4"), ("reserved", "<i4")])

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libgm_oracle.so")

DAY, WEEK, MONTH, YEAR = 0, 1, 2, 3
PERIODS = {"day": DAY, "week": WEEK, "month": MONTH, "year": YEAR}

OK, OUT_OF_BOUNDS, BAD_TIME, UNORDERED = 0, 1, 2, 3


class Range(ctypes.Structure):
    _fields_ = [("lower", ctypes.c_int64), ("upper", ctypes.c_int64),
                ("contained", ctypes.c_int32), ("pad", ctypes.c_int32)]


class PolySet(ctypes.Structure):
    _fields_ = [("n_polys", ctypes.c_int32),
                ("poly_part_off", ctypes.c_void_p), ("part_ring_off", ctypes.c_void_p),
                ("ring_vert_off", ctypes.c_void_p), ("vx", ctypes.c_void_p), ("vy", ctypes.c_void_p)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(
                os.path.join(HERE, "gm_oracle.c")):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, d, vp = ctypes.c_int64, ctypes.c_int32, ctypes.c_double, ctypes.c_void_p
        sig = {
            "gmo_d2i": (i32, [d]), "gmo_d2l": (i64, [d]),
            "gmo_z3_split": (i64, [i64]), "gmo_z3_combine": (i32, [i64]),
            "gmo_z3_apply": (i64, [i32, i32, i32]),
            "gmo_z2_split": (i64, [i64]), "gmo_z2_combine": (i32, [i64]),
            "gmo_z2_apply": (i64, [i32, i32]),
            "gmo_zdivide": (None, [ctypes.c_int, i64, i64, i64, vp, vp]),
            "gmo_zn_contains": (ctypes.c_int, [ctypes.c_int, i64, i64, i64]),
            "gmo_zn_overlaps": (ctypes.c_int, [ctypes.c_int, i64, i64, i64, i64]),
            "gmo_zranges": (i64, [ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, i64]),
            "gmo_normalize": (i32, [d, d, ctypes.c_int, d]),
            "gmo_denormalize": (d, [d, d, ctypes.c_int, i32]),
            "gmo_max_offset": (i64, [ctypes.c_int]),
            "gmo_binned_time": (ctypes.c_int, [ctypes.c_int, i64, vp, vp]),
            "gmo_binned_to_millis": (i64, [ctypes.c_int, ctypes.c_int16, i64]),
            "gmo_z3_index": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, d, d, i64, ctypes.c_int, vp]),
            "gmo_z3_invert": (None, [ctypes.c_int, ctypes.c_int, i64, vp, vp, vp]),
            "gmo_z2_index": (ctypes.c_int, [ctypes.c_int, d, d, ctypes.c_int, vp]),
            "gmo_z2_invert": (None, [ctypes.c_int, i64, vp, vp]),
            "gmo_z3_index_key_batch": (None, [ctypes.c_int, vp, vp, vp, i64, ctypes.c_int, vp, vp, vp]),
            "gmo_legacy_z3_index": (ctypes.c_int, [ctypes.c_int, d, d, i64, ctypes.c_int, vp]),
            "gmo_legacy_z3_invert": (None, [ctypes.c_int, i64, vp, vp, vp]),
            "gmo_legacy_z2_index": (ctypes.c_int, [d, d, ctypes.c_int, vp]),
            "gmo_legacy_z2_invert": (None, [i64, vp, vp]),
            "gmo_legacy_year_z3_index": (ctypes.c_int, [d, d, i64, ctypes.c_int, vp]),
            "gmo_long_binning_index": (ctypes.c_int, [i64, i64, ctypes.c_int, i64]),
            "gmo_z3_histogram": (None, [ctypes.c_int, vp, vp, vp, i64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, vp, vp, vp]),
            "gmo_z2_index_batch": (None, [vp, vp, i64, ctypes.c_int, vp, vp]),
            "gmo_z3_invert_batch": (None, [ctypes.c_int, vp, i64, vp, vp, vp]),
            "gmo_z2_invert_batch": (None, [vp, i64, vp, vp]),
            "gmo_z3_ranges": (i64, [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, vp, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, vp, i64]),
            "gmo_z2_ranges": (i64, [ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, i64]),
            "gmo_xz2_index": (ctypes.c_int, [ctypes.c_int, d, d, d, d, ctypes.c_int, vp]),
            "gmo_xz3_index": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, d, d, d, d, d, d, ctypes.c_int, vp]),
            "gmo_xz2_index_batch": (None, [ctypes.c_int, vp, vp, vp, vp, i64, ctypes.c_int, vp, vp]),
            "gmo_xz3_index_batch": (None, [ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, vp, i64, ctypes.c_int, vp, vp]),
            "gmo_xz2_ranges": (i64, [ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, vp, i64]),
            "gmo_xz3_ranges": (i64, [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, vp, i64]),
            "gmo_z3filter_in_bounds": (ctypes.c_int, [vp, ctypes.c_size_t, vp, ctypes.c_int]),
            "gmo_z2filter_in_bounds": (ctypes.c_int, [vp, ctypes.c_size_t, vp, ctypes.c_int]),
            "gmo_z3filter_scan": (i64, [vp, ctypes.c_size_t, vp, ctypes.c_int, vp, vp, i64, vp]),
            "gmo_z2filter_scan": (i64, [vp, ctypes.c_size_t, vp, i64, vp]),
            "gmo_strict_scan": (i64, [vp, vp, vp, i64, vp, ctypes.c_int, i64, i64, vp]),
            "gmo_orientation_index": (ctypes.c_int, [d, d, d, d, d, d]),
            "gmo_locate": (ctypes.c_int, [vp, ctypes.c_int, d, d]),
            "gmo_contains": (ctypes.c_int, [vp, ctypes.c_int, d, d]),
            "gmo_intersects": (ctypes.c_int, [vp, ctypes.c_int, d, d]),
            "gmo_query_scan": (i64, [vp, vp, vp, i64, vp, ctypes.c_int, i64, i64, vp, ctypes.c_int, vp]),
            "gmo_pip_join": (i64, [vp, vp, vp, i64, vp, vp, i64, ctypes.c_int]),
            "gmo_nodes_checked": (i64, []),
            "gmo_ranges_batch": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp, i64, ctypes.c_int,
                                                ctypes.c_int, vp, vp, vp, vp, vp]),
            "gmo_pip_join_ex": (i64, [vp, vp, vp, i64, vp, vp, i64, ctypes.c_int, ctypes.c_int, vp]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data if a is not None else None


# ---------------------------------------------------------------- scalar helpers

def z3_split(v): return lib().gmo_z3_split(v)
def z3_combine(z): return lib().gmo_z3_combine(z)
def z3_apply(x, y, t): return lib().gmo_z3_apply(x, y, t)
def z2_split(v): return lib().gmo_z2_split(v)
def z2_combine(z): return lib().gmo_z2_combine(z)
def z2_apply(x, y): return lib().gmo_z2_apply(x, y)
def d2i(d): return lib().gmo_d2i(d)
def normalize(mn, mx, p, x): return lib().gmo_normalize(mn, mx, p, x)
def denormalize(mn, mx, p, i): return lib().gmo_denormalize(mn, mx, p, i)
def max_offset(period): return lib().gmo_max_offset(period)


def zdivide(dims, p, rmin, rmax):
    a, b = ctypes.c_int64(), ctypes.c_int64()
    lib().gmo_zdivide(dims, p, rmin, rmax, ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def binned_time(period, ms):
    b, o = ctypes.c_int16(), ctypes.c_int64()
    st = lib().gmo_binned_time(period, ms, ctypes.byref(b), ctypes.byref(o))
    return st, b.value, o.value


def binned_to_millis(period, b, off): return lib().gmo_binned_to_millis(period, b, off)


def z3_index(x, y, t, lenient=False, period=WEEK, precision=21):
    z = ctypes.c_int64()
    st = lib().gmo_z3_index(period, precision, x, y, t, int(lenient), ctypes.byref(z))
    return st, z.value


def z3_invert(z, period=WEEK, precision=21):
    x, y, t = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    lib().gmo_z3_invert(period, precision, z, ctypes.byref(x), ctypes.byref(y), ctypes.byref(t))
    return x.value, y.value, t.value


def z2_index(x, y, lenient=False, precision=31):
    z = ctypes.c_int64()
    st = lib().gmo_z2_index(precision, x, y, int(lenient), ctypes.byref(z))
    return st, z.value


def z2_invert(z, precision=31):
    x, y = ctypes.c_double(), ctypes.c_double()
    lib().gmo_z2_invert(precision, z, ctypes.byref(x), ctypes.byref(y))
    return x.value, y.value


def xz2_index(xmin, ymin, xmax, ymax, lenient=False, g=12):
    z = ctypes.c_int64()
    st = lib().gmo_xz2_index(g, xmin, ymin, xmax, ymax, int(lenient), ctypes.byref(z))
    return st, z.value


def xz3_index(xmin, ymin, zmin, xmax, ymax, zmax, lenient=False, g=12, period=WEEK):
    z = ctypes.c_int64()
    st = lib().gmo_xz3_index(g, period, xmin, ymin, zmin, xmax, ymax, zmax, int(lenient), ctypes.byref(z))
    return st, z.value


def _ranges_call(fn, *args, cap=1 << 16):
    while True:
        out = (Range * cap)()
        n = fn(*args, ctypes.cast(out, ctypes.c_void_p), cap)
        if n < -(1 << 62):
            raise ValueError("ranges error code %d" % (n - (-(1 << 63))))
        if n < 0:
            cap = -n
            continue
        return [(out[i].lower, out[i].upper, bool(out[i].contained)) for i in range(n)]


def zranges(dims, bounds, precision=64, max_ranges=None, max_recurse=7):
    b = np.ascontiguousarray(np.asarray(bounds, dtype=np.int64).reshape(-1))
    mr = 2147483647 if max_ranges is None else max_ranges
    rec = 2147483647 if max_recurse is None else max_recurse
    return _ranges_call(lib().gmo_zranges, dims, _p(b), len(b) // 2, precision, mr, rec)


def z3_ranges(xy, t, precision=64, max_ranges=None, period=WEEK):
    a = np.ascontiguousarray(np.asarray(xy, dtype=np.float64).reshape(-1))
    tt = np.ascontiguousarray(np.asarray(t, dtype=np.int64).reshape(-1))
    mr = 2147483647 if max_ranges is None else max_ranges
    return _ranges_call(lib().gmo_z3_ranges, period, 21, _p(a), len(a) // 4, _p(tt), len(tt) // 2, precision, mr)


def z2_ranges(xy, precision=64, max_ranges=None):
    a = np.ascontiguousarray(np.asarray(xy, dtype=np.float64).reshape(-1))
    mr = 2147483647 if max_ranges is None else max_ranges
    return _ranges_call(lib().gmo_z2_ranges, 31, _p(a), len(a) // 4, precision, mr)


def nodes_checked():
    """Tree nodes the range decompositions checked on this thread since the last call."""
    return lib().gmo_nodes_checked()


def ranges_batch(kind, q, t=None, max_ranges=2000, nthreads=1, g=12, period=WEEK, lists=False):
    """Batch of single-box queries: kind "z3" (q = n x 4 boxes, t = n x 2 offsets), "xz2" (n x 4
    windows) or "xz3" (n x 6).  Returns (total merged ranges, total nodes checked); with lists=True
    also (offsets [n + 1], ranges RANGE_DTYPE) -- every query's merged list, from a second pass."""
    qa = np.ascontiguousarray(np.asarray(q, np.float64))
    ta = np.ascontiguousarray(np.asarray(t if t is not None else [0, 0], np.int64))
    k = {"z3": 3, "xz2": 12, "xz3": 13}[kind]
    nq = qa.shape[0]
    mr = 2147483647 if max_ranges is None else max_ranges
    r, nd = ctypes.c_int64(), ctypes.c_int64()
    counts = np.zeros(max(nq, 1), np.int64)
    lib().gmo_ranges_batch(k, period, g, _p(qa), _p(ta), nq, mr, nthreads, ctypes.byref(r), ctypes.byref(nd),
                           _p(counts), None, None)
    if not lists:
        return r.value, nd.value
    offs = np.zeros(nq + 1, np.int64)
    offs[1:] = np.cumsum(np.maximum(counts[:nq], 0))
    out = np.zeros(max(int(offs[-1]), 1), RANGE_DTYPE)
    lib().gmo_ranges_batch(k, period, g, _p(qa), _p(ta), nq, mr, nthreads, None, None, _p(counts), _p(offs),
                           out.ctypes.data)
    return r.value, nd.value, offs, out[:int(offs[-1])]


def xz2_ranges(queries, max_ranges=None, g=12):
    a = np.ascontiguousarray(np.asarray(queries, dtype=np.float64).reshape(-1))
    mr = 2147483647 if max_ranges is None else max_ranges
    return _ranges_call(lib().gmo_xz2_ranges, g, _p(a), len(a) // 4, mr)


def xz3_ranges(queries, max_ranges=None, g=12, period=WEEK):
    a = np.ascontiguousarray(np.asarray(queries, dtype=np.float64).reshape(-1))
    mr = 2147483647 if max_ranges is None else max_ranges
    return _ranges_call(lib().gmo_xz3_ranges, g, period, _p(a), len(a) // 6, mr)


# ---------------------------------------------------------------- batch helpers (numpy)

def z3_index_key_batch(x, y, t_ms, lenient=False, period=WEEK):
    x = np.ascontiguousarray(x, np.float64); y = np.ascontiguousarray(y, np.float64)
    t = np.ascontiguousarray(t_ms, np.int64)
    n = len(x)
    b = np.empty(n, np.int16); z = np.empty(n, np.int64); st = np.empty(n, np.uint8)
    lib().gmo_z3_index_key_batch(period, _p(x), _p(y), _p(t), n, int(lenient), _p(b), _p(z), _p(st))
    return b, z, st


def z3_histogram(x, y, t_ms, length, bin_lo, n_bins, unobserve=False, period=WEEK, present=None, counts=None,
                 tally=None):
    """Z3Histogram observe / unobserve (utils/stats/Z3Histogram.scala:101-128); returns (present, counts
    [n_bins, length], tally [skipped, outside window]), accumulating into the arrays passed in."""
    x = np.ascontiguousarray(x, np.float64); y = np.ascontiguousarray(y, np.float64)
    t = np.ascontiguousarray(t_ms, np.int64)
    present = np.zeros(n_bins, np.uint8) if present is None else present
    counts = np.zeros((n_bins, length), np.int64) if counts is None else counts
    tally = np.zeros(2, np.int64) if tally is None else tally
    lib().gmo_z3_histogram(period, _p(x), _p(y), _p(t), len(x), length, int(unobserve), bin_lo, n_bins,
                           _p(present), _p(counts), _p(tally))
    return present, counts, tally


def legacy_z3_index(x, y, t, lenient=False, period=WEEK):
    z = ctypes.c_int64()
    return lib().gmo_legacy_z3_index(period, x, y, t, int(lenient), ctypes.byref(z)), z.value


def legacy_year_z3_index(x, y, t, lenient=False):
    z = ctypes.c_int64()
    return lib().gmo_legacy_year_z3_index(x, y, t, int(lenient), ctypes.byref(z)), z.value


def legacy_z3_invert(z, period=WEEK):
    x, y, t = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    lib().gmo_legacy_z3_invert(period, z, ctypes.byref(x), ctypes.byref(y), ctypes.byref(t))
    return x.value, y.value, t.value


def legacy_z2_index(x, y, lenient=False):
    z = ctypes.c_int64()
    return lib().gmo_legacy_z2_index(x, y, int(lenient), ctypes.byref(z)), z.value


def legacy_z2_invert(z):
    x, y = ctypes.c_double(), ctypes.c_double()
    lib().gmo_legacy_z2_invert(z, ctypes.byref(x), ctypes.byref(y))
    return x.value, y.value


def long_binning_index(lo, hi, length, v):
    return lib().gmo_long_binning_index(lo, hi, length, v)


def z2_index_batch(x, y, lenient=False):
    x = np.ascontiguousarray(x, np.float64); y = np.ascontiguousarray(y, np.float64)
    n = len(x)
    z = np.empty(n, np.int64); st = np.empty(n, np.uint8)
    lib().gmo_z2_index_batch(_p(x), _p(y), n, int(lenient), _p(z), _p(st))
    return z, st


def z3_invert_batch(z, period=WEEK):
    z = np.ascontiguousarray(z, np.int64)
    n = len(z)
    x = np.empty(n); y = np.empty(n); t = np.empty(n, np.int64)
    lib().gmo_z3_invert_batch(period, _p(z), n, _p(x), _p(y), _p(t))
    return x, y, t


def z2_invert_batch(z):
    z = np.ascontiguousarray(z, np.int64)
    n = len(z)
    x = np.empty(n); y = np.empty(n)
    lib().gmo_z2_invert_batch(_p(z), n, _p(x), _p(y))
    return x, y


def xz2_index_batch(env, lenient=False, g=12):
    """XZ2SFC.index over an (n, 4) array of (xmin, ymin, xmax, ymax); returns (keys, status)."""
    env = np.asarray(env, np.float64).reshape(-1, 4)
    cols = [np.ascontiguousarray(env[:, k]) for k in range(4)]
    n = len(env)
    out = np.empty(n, np.int64); st = np.empty(n, np.uint8)
    lib().gmo_xz2_index_batch(g, *[_p(c) for c in cols], n, int(lenient), _p(out), _p(st))
    return out, st


def xz3_index_batch(env, lenient=False, g=12, period=WEEK):
    """XZ3SFC.index over an (n, 6) array of (xmin, ymin, zmin, xmax, ymax, zmax); returns (keys, status)."""
    env = np.asarray(env, np.float64).reshape(-1, 6)
    cols = [np.ascontiguousarray(env[:, k]) for k in range(6)]
    n = len(env)
    out = np.empty(n, np.int64); st = np.empty(n, np.uint8)
    lib().gmo_xz3_index_batch(g, period, *[_p(c) for c in cols], n, int(lenient), _p(out), _p(st))
    return out, st


def z3filter_scan(filter_bytes, bin_ranges, bins, zs):
    fb = np.frombuffer(bytes(filter_bytes), np.uint8).copy()
    br = np.ascontiguousarray(np.asarray(bin_ranges, np.int16).reshape(-1))
    bins = np.ascontiguousarray(bins, np.int16); zs = np.ascontiguousarray(zs, np.int64)
    m = np.empty(len(zs), np.uint8)
    c = lib().gmo_z3filter_scan(_p(fb), len(fb), _p(br) if len(br) else None, len(br) // 2, _p(bins), _p(zs),
                                len(zs), _p(m))
    if c < 0:
        raise ValueError("bad filter bytes")
    return m.astype(bool)


def z2filter_scan(filter_bytes, zs):
    fb = np.frombuffer(bytes(filter_bytes), np.uint8).copy()
    zs = np.ascontiguousarray(zs, np.int64)
    m = np.empty(len(zs), np.uint8)
    c = lib().gmo_z2filter_scan(_p(fb), len(fb), _p(zs), len(zs), _p(m))
    if c < 0:
        raise ValueError("bad filter bytes")
    return m.astype(bool)


def z3filter_in_bounds(filter_bytes, row, offset=0):
    fb = np.frombuffer(bytes(filter_bytes), np.uint8).copy()
    rb = np.frombuffer(bytes(row), np.uint8).copy()
    return bool(lib().gmo_z3filter_in_bounds(_p(fb), len(fb), _p(rb), offset))


def strict_scan(x, y, t_ms, bbox, during=None):
    x = np.ascontiguousarray(x, np.float64); y = np.ascontiguousarray(y, np.float64)
    t = np.ascontiguousarray(t_ms if t_ms is not None else np.zeros(len(x), np.int64), np.int64)
    bb = np.ascontiguousarray(bbox, np.float64)
    m = np.empty(len(x), np.uint8)
    lo, hi = during if during is not None else (0, 0)
    lib().gmo_strict_scan(_p(x), _p(y), _p(t), len(x), _p(bb), int(during is not None), lo, hi, _p(m))
    return m.astype(bool)


def query_scan(x, y, t_ms=None, bbox=None, during=None, polys=None, op=0):
    """bbox AND during AND (OR over polys of INTERSECTS (op 1) / CONTAINS (op 2)); polys is an
    OraclePolySet.  Returns the boolean match column."""
    x = np.ascontiguousarray(x, np.float64); y = np.ascontiguousarray(y, np.float64)
    t = np.ascontiguousarray(t_ms if t_ms is not None else np.zeros(len(x), np.int64), np.int64)
    bb = np.ascontiguousarray(bbox, np.float64) if bbox is not None else None
    m = np.empty(len(x), np.uint8)
    lo, hi = during if during is not None else (0, 0)
    ps = ctypes.byref(polys.c) if polys is not None else None
    lib().gmo_query_scan(_p(x), _p(y), _p(t), len(x), _p(bb), int(during is not None), lo, hi, ps, op, _p(m))
    return m.astype(bool)


class OraclePolySet:
    """Keeps numpy CSR arrays alive for the C gmo_polyset view."""

    def __init__(self, poly_part_off, part_ring_off, ring_vert_off, vx, vy):
        self.arrs = [np.ascontiguousarray(a, np.int32) for a in (poly_part_off, part_ring_off, ring_vert_off)]
        self.vx = np.ascontiguousarray(vx, np.float64)
        self.vy = np.ascontiguousarray(vy, np.float64)
        self.c = PolySet(len(self.arrs[0]) - 1, _p(self.arrs[0]), _p(self.arrs[1]), _p(self.arrs[2]),
                         _p(self.vx), _p(self.vy))

    def contains(self, poly, x, y):
        return bool(lib().gmo_contains(ctypes.byref(self.c), poly, x, y))

    def locate(self, poly, x, y):
        return lib().gmo_locate(ctypes.byref(self.c), poly, x, y)

    def intersects(self, poly, x, y):
        return bool(lib().gmo_intersects(ctypes.byref(self.c), poly, x, y))

    def join(self, px, py, nthreads=1, predicate="st_contains", with_edges=False):
        """(point ids, polygon ids) of the join; with_edges also returns E_c, the candidate edges."""
        px = np.ascontiguousarray(px, np.float64); py = np.ascontiguousarray(py, np.float64)
        op = {"st_contains": 2, "st_within": 2, "st_intersects": 1, "st_covers": 1}[predicate]
        cap = max(1024, len(px) // 4)
        ec = ctypes.c_int64()
        while True:
            pt = np.empty(cap, np.int64); pl = np.empty(cap, np.int32)
            n = lib().gmo_pip_join_ex(ctypes.byref(self.c), _p(px), _p(py), len(px), _p(pt), _p(pl), cap, nthreads,
                                      op, ctypes.byref(ec))
            if n < 0:
                cap = -n
                continue
            if with_edges:
                return pt[:n].copy(), pl[:n].copy(), ec.value
            return pt[:n].copy(), pl[:n].copy()


def orientation_index(p1x, p1y, p2x, p2y, qx, qy):
    return lib().gmo_orientation_index(p1x, p1y, p2x, p2y, qx, qy)


def zn_contains(dims, rmin, rmax, v): return bool(lib().gmo_zn_contains(dims, rmin, rmax, v))
def zn_overlaps(dims, rmin, rmax, vmin, vmax): return bool(lib().gmo_zn_overlaps(dims, rmin, rmax, vmin, vmax))


# ---------------------------------------------------------------- Arrow geometry vectors (8(f).2)
# Per-row restatement of reading geomesa-arrow-jts vectors: tuple order [y, x] unless flipAxisOrder
# (impl/AbstractPointVector.java:52-79), shell-first rings (impl/AbstractPolygonVector.java:56-84),
# and the JTS 1.20 envelope rules of Geometry.getEnvelopeInternal (Envelope.expandToInclude: a null
# envelope reads back as (0, -1, 0, -1); Polygon -> its shell's; collections -> union of parts').
# Pure Python loops: small cases only.

NULL_GEOM = 4
_DEPTH = {"point": 0, "linestring": 1, "multipoint": 1, "polygon": 2, "multilinestring": 2, "multipolygon": 3}


def arrow_rows(arr, kind, flip_axis=False):
    """pyarrow geometry array -> per-row nested lists of (x, y) (None for a null slot)."""
    def xy(t):
        return (t[0], t[1]) if flip_axis else (t[1], t[0])

    def conv(v, depth):
        return xy(v) if depth == 0 else [conv(c, depth - 1) for c in v]
    return [None if v is None else conv(v, _DEPTH[kind]) for v in arr.to_pylist()]


def _env_expand(e, x, y):
    if e is None:
        return [x, x, y, y]
    if x < e[0]: e[0] = x
    if x > e[1]: e[1] = x
    if y < e[2]: e[2] = y
    if y > e[3]: e[3] = y
    return e


def _env_merge(e, o):
    if o is None:
        return e
    if e is None:
        return list(o)
    return _env_expand(_env_expand(e, o[0], o[2]), o[1], o[3])


def jts_envelope(row, kind):
    """(minx, miny, maxx, maxy) of a non-null row, JTS null envelope -> (0, 0, -1, -1)."""
    def seq(ts):
        e = None
        for x, y in ts:
            e = _env_expand(e, x, y)
        return e
    if kind == "point":
        e = seq([row])
    elif kind in ("linestring", "multipoint"):
        e = seq(row)
    elif kind == "polygon":
        e = seq(row[0]) if row else None
    elif kind == "multilinestring":
        e = None
        for line in row:
            e = _env_merge(e, seq(line))
    else:
        e = None
        for poly in row:
            if poly:
                e = _env_merge(e, seq(poly[0]))
    if e is None:
        return (0.0, 0.0, -1.0, -1.0)
    return (e[0], e[2], e[1], e[3])


def _times(dtg, n):
    if dtg is None:
        return [0] * n
    vals = dtg.cast("int64").to_pylist() if hasattr(dtg, "cast") else list(dtg)
    return [0 if v is None else int(v) for v in vals]


def arrow_z3_keys(arr, dtg=None, lenient=False, period=WEEK, flip_axis=False):
    """Z3IndexKeySpace.toIndexKey (Z3IndexKeySpace.scala:63-76) per Arrow row."""
    rows = arrow_rows(arr, "point", flip_axis)
    ts = _times(dtg, len(rows))
    b = np.zeros(len(rows), np.int16); z = np.zeros(len(rows), np.int64); st = np.zeros(len(rows), np.uint8)
    for i, (r, t) in enumerate(zip(rows, ts)):
        if r is None:
            st[i] = NULL_GEOM
            continue
        bb, zz, s = z3_index_key_batch([r[0]], [r[1]], [t], lenient, period)
        b[i], z[i], st[i] = bb[0], zz[0], s[0]
    return b, z, st


def arrow_z2_keys(arr, lenient=False, flip_axis=False):
    rows = arrow_rows(arr, "point", flip_axis)
    z = np.zeros(len(rows), np.int64); st = np.zeros(len(rows), np.uint8)
    for i, r in enumerate(rows):
        if r is None:
            st[i] = NULL_GEOM
            continue
        st[i], z[i] = z2_index(r[0], r[1], lenient)
    return z, st


def arrow_xz2_keys(arr, kind, g=12, lenient=False, flip_axis=False):
    """XZ2IndexKeySpace.toIndexKey (XZ2IndexKeySpace.scala:48-58) per Arrow row."""
    rows = arrow_rows(arr, kind, flip_axis)
    z = np.zeros(len(rows), np.int64); st = np.zeros(len(rows), np.uint8)
    for i, r in enumerate(rows):
        if r is None:
            st[i] = NULL_GEOM
            continue
        st[i], z[i] = xz2_index(*jts_envelope(r, kind), lenient=lenient, g=g)
        if st[i]:
            z[i] = 0
    return z, st


def arrow_xz3_keys(arr, dtg, kind, g=12, period=WEEK, lenient=False, flip_axis=False):
    """XZ3IndexKeySpace.toIndexKey (XZ3IndexKeySpace.scala:60-76) per Arrow row."""
    rows = arrow_rows(arr, kind, flip_axis)
    ts = _times(dtg, len(rows))
    b = np.zeros(len(rows), np.int16); z = np.zeros(len(rows), np.int64); st = np.zeros(len(rows), np.uint8)
    for i, (r, t) in enumerate(zip(rows, ts)):
        if r is None:
            st[i] = NULL_GEOM
            continue
        s, bb, off = binned_time(period, t)
        if s:
            st[i] = s
            continue
        x0, y0, x1, y1 = jts_envelope(r, kind)
        s, zz = xz3_index(x0, y0, float(off), x1, y1, float(off), lenient=lenient, g=g, period=period)
        st[i] = s
        if not s:
            b[i], z[i] = bb, zz
    return b, z, st


# ---------------------------------------------------------------- key-range partition (multi-GPU ingest)
def table_key_u64(shard, bins, zs):
    """(key_hi, key_lo) uint64 of (shard u8 or None, bin i16, z i64): the [shard][bin BE16][z BE64] row-key
    byte order (Z3IndexKeySpace.scala:81-92) as an unsigned pair."""
    hi = np.asarray(bins).astype(np.int64).astype(np.uint64) & np.uint64(0xffff)
    if shard is not None:
        hi = hi | (np.asarray(shard).astype(np.uint64) << np.uint64(16))
    return hi, np.asarray(zs).astype(np.int64).view(np.uint64)


def key_partition(shard, bins, zs, sp_hi, sp_lo):
    """The definition gm_key_partition implements: destination = number of splitters <= key (a key equal
    to a splitter opens the upper range, the tablet split semantics of a sorted store); rows grouped by
    destination, stable.  Returns (order, counts): the input rows in output order and the per-destination
    row counts."""
    hi, lo = table_key_u64(shard, bins, zs)
    sp_hi = np.asarray(sp_hi, np.uint64)
    sp_lo = np.asarray(sp_lo, np.uint64)
    dest = np.zeros(len(hi), np.int64)
    for h, l_ in zip(sp_hi, sp_lo):
        dest += (hi > h) | ((hi == h) & (lo >= l_))
    order = np.argsort(dest, kind="stable")
    return order, np.bincount(dest, minlength=len(sp_hi) + 1).astype(np.int64)


# ---------------------------------------------------------------- the XZ full filter (full-scan restatement)
def envelope_scan(xmin, ymin, xmax, ymax, boxes, t_ms=None, interval=None):
    """Mask of features whose envelope intersects any box (JTS Envelope.intersects: inclusive, a null
    envelope -- max < min -- never intersects) AND, with an interval, whose dtg lies in (lo, hi) (FastDuring,
    exclusive; FastTemporalOperator.scala:116-129): the full filter the XZ key spaces apply
    (XZ2IndexKeySpace.scala:122-125, XZ3IndexKeySpace.scala:247-250), evaluated on every feature."""
    xmin, ymin, xmax, ymax = (np.asarray(c, np.float64) for c in (xmin, ymin, xmax, ymax))
    ok = np.zeros(len(xmin), bool)
    valid = ~((xmax < xmin) | (ymax < ymin))
    for (bx0, by0, bx1, by1) in boxes:
        if bx1 < bx0 or by1 < by0:
            continue
        ok |= valid & ~((bx0 > xmax) | (bx1 < xmin) | (by0 > ymax) | (by1 < ymin))
    if interval is not None:
        t = np.asarray(t_ms, np.int64)
        ok &= (t > interval[0]) & (t < interval[1])
    return ok
