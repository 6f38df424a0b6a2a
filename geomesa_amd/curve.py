"""Space-filling curves: the batch form of geomesa-z3's curve API, executed by libgeomesa_hip.

Mirrors the reference Scala surface (paths relative to
geomesa-z3/src/main/scala/org/locationtech/geomesa/):

  * ``Z3SFC(period, precision=21)``  -- curve/Z3SFC.scala:21-100
  * ``Z2SFC(precision=31)``          -- curve/Z2SFC.scala:14-53
  * ``XZ2SFC(g)`` / ``XZ3SFC(g, period)`` -- curve/XZ2SFC.scala, curve/XZ3SFC.scala
  * ``BinnedTime`` / ``TimePeriod``   -- curve/BinnedTime.scala

Every ``index``/``invert`` takes columns (torch tensors on the GPU, or anything numpy can read,
which is then copied to the GPU) and returns GPU tensors.  As in the Scala code, a non-lenient
``index`` raises ``IllegalArgumentException`` for the first out-of-bounds element, and BinnedTime
raises for times before 1970 or past the period's max date even when lenient.

``ranges`` returns a list of ``IndexRange`` per query (batched on the GPU).
"""
import ctypes
from collections import namedtuple

import numpy as np

from . import _lib
from ._lib import check, ptr


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException raised by the Scala require(...) calls."""


class TimePeriod:
    """TimePeriod enumeration (curve/BinnedTime.scala:283-291)."""
    Day, Week, Month, Year = 0, 1, 2, 3
    _names = {"day": 0, "week": 1, "month": 2, "year": 3}

    @classmethod
    def of(cls, p):
        if isinstance(p, str):
            return cls._names[p.lower()]
        if p in (0, 1, 2, 3):
            return int(p)
        raise IllegalArgumentException("unknown time period %r" % (p,))


IndexRange = namedtuple("IndexRange", ["lower", "upper", "contained"])  # package.scala:45-76


def CoveredRange(lower, upper):
    return IndexRange(lower, upper, True)


def OverlappingRange(lower, upper):
    return IndexRange(lower, upper, False)


def max_offset(period):
    """BinnedTime.maxOffset (curve/BinnedTime.scala:148-156)."""
    return {0: 86400000, 1: 604800, 2: 86400 * 31, 3: 1440 * 366 + 10}[TimePeriod.of(period)]


class NormalizedDimension:
    """BitNormalizedDimension constants (curve/NormalizedDimension.scala:56-72)."""

    def __init__(self, mn, mx, precision):
        if not (0 < precision < 32):
            raise IllegalArgumentException("Precision (bits) must be in [1,31]")
        self.min = float(mn)
        self.max = float(mx)
        self.precision = precision
        bins = 1 << precision
        self.normalizer = bins / (self.max - self.min)
        self.denormalizer = (self.max - self.min) / bins
        self.maxIndex = bins - 1

    # host-side scalar forms (used by query planning, e.g. Z3Filter construction)
    def normalize(self, x):
        import math
        if x >= self.max:
            return self.maxIndex
        v = math.floor((x - self.min) * self.normalizer)
        if v != v:
            return 0
        return int(max(-2147483648, min(2147483647, v)))

    def denormalize(self, i):
        if i >= self.maxIndex:
            return self.min + (self.maxIndex + 0.5) * self.denormalizer
        return self.min + (i + 0.5) * self.denormalizer


def _jvm_to_int(v):
    """Double.toInt: NaN -> 0, saturating at Int.MinValue / Int.MaxValue."""
    if v != v:
        return 0
    if v >= 2147483647:
        return 2147483647
    if v <= -2147483648:
        return -2147483648
    return int(v)


class SemiNormalizedDimension:
    """Legacy SemiNormalizedDimension (curve/NormalizedDimension.scala:83-87): ceil-based, maxIndex =
    precision (2^21 - 1 or 2^20 - 1).  Host scalar forms for query planning on legacy indices."""

    def __init__(self, mn, mx, precision):
        self.min = float(mn)
        self.max = float(mx)
        self.precision = int(precision)
        self.maxIndex = int(precision)

    def normalize(self, x):   # math.ceil((x - min) / (max - min) * precision).toInt   (:85)
        import math
        v = (float(x) - self.min) / (self.max - self.min) * float(self.precision)
        if v != v or v in (float("inf"), float("-inf")):
            return _jvm_to_int(v)
        return _jvm_to_int(math.ceil(v))

    def denormalize(self, i):   # :86
        if i == 0:
            return self.min
        return (i - 0.5) * (self.max - self.min) / float(self.precision) + self.min


# ------------------------------------------------------------------------------ column helpers

def _torch():
    import torch
    return torch


def _dev_col(a, dtype):
    """Return a contiguous GPU tensor of `dtype` for column `a` (no copy if already one)."""
    torch = _torch()
    ctx = _lib.context()
    dev = torch.device("cuda", ctx.device)
    if isinstance(a, torch.Tensor):
        t = a
        if t.device != dev:
            t = t.to(dev)
        if t.dtype != dtype:
            t = t.to(dtype)
        return t.contiguous()
    arr = np.ascontiguousarray(np.asarray(a), dtype={torch.float64: np.float64, torch.int64: np.int64,
                                                     torch.int16: np.int16}[dtype])
    return torch.from_numpy(arr).to(dev)


def _summary():
    return _lib.BatchStatus()


def _raise_first(st, what, status=None):
    if st.n_errors > 0:
        code = st.first_code
        if code == _lib.GM_ST_BAD_TIME:
            msg = "Date exceeds indexable bounds (element %d)" % st.first_index
        elif code == _lib.GM_ST_UNORDERED:
            msg = "Bounds must be ordered (element %d)" % st.first_index
        else:
            msg = "Value(s) out of bounds (element %d)" % st.first_index
        raise IllegalArgumentException("%s: %s" % (what, msg))


class BinnedTime:
    """BinnedTime.timeToBinnedTime(period) over a column of epoch millis (curve/BinnedTime.scala:73-86)."""

    @staticmethod
    def time_to_binned_time(period, t_ms, status=False):
        torch = _torch()
        p = TimePeriod.of(period)
        t = _dev_col(t_ms, torch.int64)
        n = t.numel()
        ctx = _lib.context()
        b = torch.empty(n, dtype=torch.int16, device=t.device)
        o = torch.empty(n, dtype=torch.int64, device=t.device)
        s = torch.empty(n, dtype=torch.uint8, device=t.device) if status else None
        st = _summary()
        check(ctx.lib.gm_binned_time(ctx.handle, ptr(t), n, p, ptr(b), ptr(o), ptr(s), ctypes.byref(st)),
              "gm_binned_time")
        if status:
            return b, o, s
        _raise_first(st, "BinnedTime")
        return b, o


class Z3SFC:
    """Z3 space filling curve (curve/Z3SFC.scala:21-100)."""

    _cache = {}

    def __new__(cls, period=TimePeriod.Week, precision=21):
        key = (TimePeriod.of(period), precision)
        if key not in cls._cache:
            if not (0 < precision < 22):
                raise IllegalArgumentException("Precision (bits) per dimension must be in [1,21]")
            o = super().__new__(cls)
            o.period, o.precision = key
            o.lon = NormalizedDimension(-180.0, 180.0, precision)
            o.lat = NormalizedDimension(-90.0, 90.0, precision)
            o.time = NormalizedDimension(0.0, float(max_offset(o.period)), precision)
            o.wholePeriod = [(int(o.time.min), int(o.time.max))]
            cls._cache[key] = o
        return cls._cache[key]

    def index(self, x, y, t, lenient=False, status=False):
        """Z3SFC.index (Z3SFC.scala:37-52); t = offset within the period."""
        torch = _torch()
        x = _dev_col(x, torch.float64); y = _dev_col(y, torch.float64); t = _dev_col(t, torch.int64)
        n = x.numel()
        ctx = _lib.context()
        z = torch.empty(n, dtype=torch.int64, device=x.device)
        s = torch.empty(n, dtype=torch.uint8, device=x.device) if status else None
        st = _summary()
        check(ctx.lib.gm_z3_index(ctx.handle, ptr(x), ptr(y), ptr(t), n, self.period, self.precision,
                                  int(bool(lenient)), ptr(z), ptr(s), ctypes.byref(st)), "gm_z3_index")
        if status:
            return z, s
        _raise_first(st, "Z3SFC.index")
        return z

    def index_keys(self, x, y, t_ms, lenient=False, status=False):
        """Z3IndexKeySpace.toIndexKey's (bin, z) for epoch-millis times (Z3IndexKeySpace.scala:71-76)."""
        torch = _torch()
        if self.precision != 21:
            raise IllegalArgumentException("index keys use the standard 21-bit curve")
        x = _dev_col(x, torch.float64); y = _dev_col(y, torch.float64); t = _dev_col(t_ms, torch.int64)
        n = x.numel()
        ctx = _lib.context()
        b = torch.empty(n, dtype=torch.int16, device=x.device)
        z = torch.empty(n, dtype=torch.int64, device=x.device)
        s = torch.empty(n, dtype=torch.uint8, device=x.device) if status else None
        st = _summary()
        check(ctx.lib.gm_z3_index_key(ctx.handle, ptr(x), ptr(y), ptr(t), n, self.period, int(bool(lenient)),
                                      ptr(b), ptr(z), ptr(s), ctypes.byref(st)), "gm_z3_index_key")
        if status:
            return b, z, s
        _raise_first(st, "Z3IndexKeySpace.toIndexKey")
        return b, z

    def invert(self, z):
        """Z3SFC.invert (Z3SFC.scala:54-57) -> (x, y, t)."""
        torch = _torch()
        z = _dev_col(z, torch.int64)
        n = z.numel()
        ctx = _lib.context()
        x = torch.empty(n, dtype=torch.float64, device=z.device)
        y = torch.empty(n, dtype=torch.float64, device=z.device)
        t = torch.empty(n, dtype=torch.int64, device=z.device)
        check(ctx.lib.gm_z3_invert(ctx.handle, ptr(z), n, self.period, self.precision, ptr(x), ptr(y), ptr(t)),
              "gm_z3_invert")
        return x, y, t

    def ranges(self, xy, t, precision=64, max_ranges=None):
        """Z3SFC.ranges (Z3SFC.scala:59-67) for one query."""
        return self.ranges_batch([(xy, t)], precision, max_ranges)[0]

    def ranges_batch(self, queries, precision=64, max_ranges=None, max_recurse=None):
        """Batched Z3SFC.ranges: queries = [(xy boxes, t intervals)], one ZN.zranges per query."""
        from . import ranges as R
        return R.z3_ranges(self, queries, precision, max_ranges, max_recurse)


class Z2SFC:
    """Z2 space filling curve (curve/Z2SFC.scala:14-53); Z2SFC() is the 31-bit object."""

    _cache = {}

    def __new__(cls, precision=31):
        if precision not in cls._cache:
            o = super().__new__(cls)
            o.precision = precision
            o.lon = NormalizedDimension(-180.0, 180.0, precision)
            o.lat = NormalizedDimension(-90.0, 90.0, precision)
            cls._cache[precision] = o
        return cls._cache[precision]

    def index(self, x, y, lenient=False, status=False):
        torch = _torch()
        x = _dev_col(x, torch.float64); y = _dev_col(y, torch.float64)
        n = x.numel()
        ctx = _lib.context()
        z = torch.empty(n, dtype=torch.int64, device=x.device)
        s = torch.empty(n, dtype=torch.uint8, device=x.device) if status else None
        st = _summary()
        check(ctx.lib.gm_z2_index(ctx.handle, ptr(x), ptr(y), n, self.precision, int(bool(lenient)), ptr(z),
                                  ptr(s), ctypes.byref(st)), "gm_z2_index")
        if status:
            return z, s
        _raise_first(st, "Z2SFC.index")
        return z

    def invert(self, z):
        torch = _torch()
        z = _dev_col(z, torch.int64)
        n = z.numel()
        ctx = _lib.context()
        x = torch.empty(n, dtype=torch.float64, device=z.device)
        y = torch.empty(n, dtype=torch.float64, device=z.device)
        check(ctx.lib.gm_z2_invert(ctx.handle, ptr(z), n, self.precision, ptr(x), ptr(y)), "gm_z2_invert")
        return x, y

    def ranges(self, xy, precision=64, max_ranges=None):
        return self.ranges_batch([xy], precision, max_ranges)[0]

    def ranges_batch(self, queries, precision=64, max_ranges=None, max_recurse=None):
        from . import ranges as R
        return R.z2_ranges(self, queries, precision, max_ranges, max_recurse)


class XZ2SFC:
    """XZ2 curve (curve/XZ2SFC.scala:24-417); XZ2SFC(g) caches per g like the Scala object."""

    _cache = {}

    def __new__(cls, g=12):
        if g not in cls._cache:
            o = super().__new__(cls)
            o.g = int(g)
            cls._cache[g] = o
        return cls._cache[g]

    def index(self, xmin, ymin, xmax, ymax, lenient=False, status=False):
        torch = _torch()
        cols = [_dev_col(c, torch.float64) for c in (xmin, ymin, xmax, ymax)]
        n = cols[0].numel()
        ctx = _lib.context()
        out = torch.empty(n, dtype=torch.int64, device=cols[0].device)
        s = torch.empty(n, dtype=torch.uint8, device=out.device) if status else None
        st = _summary()
        check(ctx.lib.gm_xz2_index(ctx.handle, *[ptr(c) for c in cols], n, self.g, int(bool(lenient)), ptr(out),
                                   ptr(s), ctypes.byref(st)), "gm_xz2_index")
        if status:
            return out, s
        _raise_first(st, "XZ2SFC.index")
        return out

    def ranges(self, queries, max_ranges=None):
        """XZ2SFC.ranges(Seq[window], maxRanges) (XZ2SFC.scala:130-137) for one OR'd window set."""
        return self.ranges_batch([queries], max_ranges)[0]

    def ranges_batch(self, queries, max_ranges=None):
        from . import ranges as R
        return R.xz2_ranges(self, queries, max_ranges)


class XZ3SFC:
    """XZ3 curve (curve/XZ3SFC.scala:26-465); z = time offset in the period."""

    _cache = {}

    def __new__(cls, g=12, period=TimePeriod.Week):
        key = (int(g), TimePeriod.of(period))
        if key not in cls._cache:
            o = super().__new__(cls)
            o.g, o.period = key
            o.zBounds = (0.0, float(max_offset(o.period)))
            cls._cache[key] = o
        return cls._cache[key]

    def index(self, xmin, ymin, zmin, xmax, ymax, zmax, lenient=False, status=False):
        torch = _torch()
        cols = [_dev_col(c, torch.float64) for c in (xmin, ymin, zmin, xmax, ymax, zmax)]
        n = cols[0].numel()
        ctx = _lib.context()
        out = torch.empty(n, dtype=torch.int64, device=cols[0].device)
        s = torch.empty(n, dtype=torch.uint8, device=out.device) if status else None
        st = _summary()
        check(ctx.lib.gm_xz3_index(ctx.handle, *[ptr(c) for c in cols], n, self.g, self.period,
                                   int(bool(lenient)), ptr(out), ptr(s), ctypes.byref(st)), "gm_xz3_index")
        if status:
            return out, s
        _raise_first(st, "XZ3SFC.index")
        return out

    def ranges(self, queries, max_ranges=None):
        return self.ranges_batch([queries], max_ranges)[0]

    def ranges_batch(self, queries, max_ranges=None):
        from . import ranges as R
        return R.xz3_ranges(self, queries, max_ranges)


class _LegacyBase:
    @staticmethod
    def _run_index(fn, cols, n, extra, lenient, status, what):
        torch = _torch()
        ctx = _lib.context()
        z = torch.empty(n, dtype=torch.int64, device=cols[0].device)
        s = torch.empty(n, dtype=torch.uint8, device=cols[0].device) if status else None
        st = _summary()
        check(getattr(ctx.lib, fn)(ctx.handle, *[ptr(c) for c in cols], n, *extra, int(bool(lenient)), ptr(z), ptr(s),
                                   ctypes.byref(st)), fn)
        if status:
            return z, s
        _raise_first(st, what)
        return z


class LegacyZ3SFC(_LegacyBase):
    """LegacyZ3SFC(period) (curve/LegacyZ3SFC.scala:18-49): semi-normalized dimensions, kept for old data."""
    LEGACY_Z3, LEGACY_YEAR_Z3 = 0, 1

    def __init__(self, period=TimePeriod.Week):
        self.period = TimePeriod.of(period)
        self.curve = self.LEGACY_Z3
        # LegacyZ3Dimensions (LegacyZ3SFC.scala:46-51): host planning forms of the dimensions
        self.precision = 21
        self.lon = SemiNormalizedDimension(-180.0, 180.0, (1 << 21) - 1)
        self.lat = SemiNormalizedDimension(-90.0, 90.0, (1 << 21) - 1)
        self.time = SemiNormalizedDimension(0.0, float(max_offset(self.period)), (1 << 20) - 1)
        self.wholePeriod = [(int(self.time.min), int(self.time.max))]   # Z3SFC.wholePeriod (Z3SFC.scala:27)

    def index(self, x, y, t, lenient=False, status=False):
        torch = _torch()
        cols = [_dev_col(x, torch.float64), _dev_col(y, torch.float64), _dev_col(t, torch.int64)]
        return self._run_index("gm_legacy_z3_index", cols, cols[0].numel(), (self.curve, self.period), lenient,
                               status, type(self).__name__ + ".index")

    def index_keys(self, x, y, t_ms, lenient=False, status=False):
        """Z3IndexKeySpaceV4's (bin, z) (legacy/Z3IndexV4.scala:44-51 over Z3IndexKeySpace.scala:71-76):
        BinnedTime (raises for out-of-range dates even when lenient), then this curve's index."""
        if status:
            raise IllegalArgumentException("per-element status is not offered for the legacy key space")
        bins, off = BinnedTime.time_to_binned_time(self.period, t_ms)
        return bins, self.index(x, y, off, lenient=lenient)

    def ranges(self, xy, t, precision=64, max_ranges=None):
        """Z3SFC.ranges (Z3SFC.scala:59-67), which LegacyZ3SFC inherits, for one query."""
        return self.ranges_batch([(xy, t)], precision, max_ranges)[0]

    def ranges_batch(self, queries, precision=64, max_ranges=None, max_recurse=None):
        """Z3SFC.ranges as LegacyZ3SFC inherits it (Z3SFC.scala:59-67): per (box, interval) a
        ZRange(index(xmin, ymin, tmin), index(xmax, ymax, tmax)) through THIS curve's (legacy,
        non-lenient) index, then Z3.zranges with Z3SFC.MaxRecursion = Int.MaxValue (Z3SFC.scala:72).
        Corners are keyed on the device (gm_legacy_z3_index), the walk is gm_zranges."""
        from . import ranges as R
        lo_x, lo_y, lo_t, hi_x, hi_y, hi_t, counts = [], [], [], [], [], [], []
        for (bxs, ts) in queries:
            k = 0
            for (xmin, ymin, xmax, ymax) in bxs:
                for (tmin, tmax) in ts:
                    lo_x.append(float(xmin)); lo_y.append(float(ymin)); lo_t.append(int(tmin))
                    hi_x.append(float(xmax)); hi_y.append(float(ymax)); hi_t.append(int(tmax))
                    k += 1
            counts.append(k)
        bounds = [[] for _ in queries]
        if lo_x:
            zlo = self.index(lo_x, lo_y, lo_t).cpu().tolist()   # require(...) raises like the Scala index
            zhi = self.index(hi_x, hi_y, hi_t).cpu().tolist()
            k = 0
            for q, c in enumerate(counts):
                bounds[q] = list(zip(zlo[k:k + c], zhi[k:k + c]))
                k += c
        return R.zranges(3, bounds, precision, max_ranges, (1 << 31) - 1 if max_recurse is None else max_recurse)

    def invert(self, z):
        torch = _torch()
        if self.curve != self.LEGACY_Z3:
            raise IllegalArgumentException("invert is only defined here for LegacyZ3SFC")
        z = _dev_col(z, torch.int64)
        n = z.numel()
        ctx = _lib.context()
        x = torch.empty(n, dtype=torch.float64, device=z.device)
        y = torch.empty(n, dtype=torch.float64, device=z.device)
        t = torch.empty(n, dtype=torch.int64, device=z.device)
        check(ctx.lib.gm_legacy_z3_invert(ctx.handle, ptr(z), n, self.curve, self.period, ptr(x), ptr(y), ptr(t)),
              "gm_legacy_z3_invert")
        return x, y, t


class LegacyYearZ3SFC(LegacyZ3SFC):
    """LegacyYearZ3SFC (curve/LegacyYearZ3SFC.scala:17-46): 21-bit curve, legacy 52-week time max."""

    def __init__(self):
        super().__init__(TimePeriod.Year)
        self.curve = self.LEGACY_YEAR_Z3


class LegacyZ2SFC(_LegacyBase):
    """LegacyZ2SFC (curve/LegacyZ2SFC.scala:14-26)."""

    def index(self, x, y, lenient=False, status=False):
        torch = _torch()
        cols = [_dev_col(x, torch.float64), _dev_col(y, torch.float64)]
        return self._run_index("gm_legacy_z2_index", cols, cols[0].numel(), (), lenient, status, "LegacyZ2SFC.index")

    def invert(self, z):
        torch = _torch()
        z = _dev_col(z, torch.int64)
        n = z.numel()
        ctx = _lib.context()
        x = torch.empty(n, dtype=torch.float64, device=z.device)
        y = torch.empty(n, dtype=torch.float64, device=z.device)
        check(ctx.lib.gm_legacy_z2_invert(ctx.handle, ptr(z), n, ptr(x), ptr(y)), "gm_legacy_z2_invert")
        return x, y
