"""Z3 / Z2 index key spaces: the callers of the hot path (query planning + key layout).

Mirrors geomesa-index-api/src/main/scala/org/locationtech/geomesa/index/index/z3/Z3IndexKeySpace.scala
(toIndexKey :63-95, getIndexValues :97-159, getRanges :161-194, getRangeBytes :196-238) and the
interval extraction of geomesa-filter's FilterHelper.extractIntervals (FilterHelper.scala:146-190)
for the bbox / during / between / comparison predicates on this path.  Planning is per query and
runs on the host (as it does in the reference client); the per-row work -- key encoding, range
decomposition batches and filter scans -- runs on the GPU through libgeomesa_hip.
"""
import math
from dataclasses import dataclass, field

import numpy as np

from .curve import (BinnedTime, IllegalArgumentException, LegacyZ3SFC, TimePeriod, XZ2SFC, XZ3SFC, Z2SFC, Z3SFC,
                    max_offset)

SHORT_MAX = 32767
WHOLE_WORLD = (-180.0, -90.0, 180.0, 90.0)


@dataclass
class Bounds:
    """geomesa-filter Bounds[Date] in epoch millis; None = unbounded side."""
    lower: int = None
    upper: int = None
    lower_inclusive: bool = True
    upper_inclusive: bool = True

    @property
    def is_bounded_both_sides(self):
        return self.lower is not None and self.upper is not None


def during(lo_ms, hi_ms):
    """ECQL `dtg DURING lo/hi`: exclusive at both ends (FastTemporalOperator.scala:116-129)."""
    return Bounds(lo_ms, hi_ms, False, False)


def between(lo_ms, hi_ms):
    """ECQL `dtg BETWEEN lo AND hi`: inclusive at both ends."""
    return Bounds(lo_ms, hi_ms, True, True)


def _round_up(ms):    # roundSecondsUp: plusSeconds(1).withNano(0)   (FilterHelper.scala:182)
    return (ms + 1000) // 1000 * 1000


def _round_down(ms):  # roundSecondsDown (FilterHelper.scala:184-187)
    return ms - 1000 if ms % 1000 == 0 else ms // 1000 * 1000


def extract_interval(b, handle_exclusive_bounds=True):
    """FilterHelper.extractIntervals for one Bounds (FilterHelper.scala:146-167)."""
    def create(v, incl, rnd, round_excl):
        if v is None:
            return None, incl
        if round_excl and not incl:
            return rnd(v), True
        return v, incl
    if (not handle_exclusive_bounds or b.lower is None or b.upper is None or
            (b.lower_inclusive and b.upper_inclusive)):
        lo, li = create(b.lower, b.lower_inclusive, _round_up, handle_exclusive_bounds)
        hi, hi_i = create(b.upper, b.upper_inclusive, _round_down, handle_exclusive_bounds)
    else:
        margin = 1000 if (b.lower_inclusive or b.upper_inclusive) else 2000
        rnd = b.upper - b.lower > margin
        lo, li = create(b.lower, b.lower_inclusive, _round_up, rnd)
        hi, hi_i = create(b.upper, b.upper_inclusive, _round_down, rnd)
    return Bounds(lo, hi, li, hi_i)


def _epoch_ms_max(period):
    """BinnedTime.maxDate(period) in epoch millis (exclusive) (BinnedTime.scala:62-65,164-171)."""
    p = TimePeriod.of(period)
    if p == TimePeriod.Day:
        return 32768 * 86400000
    if p == TimePeriod.Week:
        return 32768 * 604800000
    import datetime
    if p == TimePeriod.Month:
        y, m = divmod(1970 * 12 + 32768, 12)
        d = datetime.date(y, m + 1, 1)
    else:
        d = datetime.date(1970 + 32768, 1, 1) if 1970 + 32768 <= 9999 else None
        if d is None:  # beyond python's date range: days_from_civil
            return _days_from_civil(1970 + 32768, 1, 1) * 86400000
    return _days_from_civil(d.year, d.month, d.day) * 86400000


def _days_from_civil(y, m, d):
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    doy = (153 * (m - 3 if m > 2 else m + 9) + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def _civil_from_days(z):
    z += 719468
    era = (z if z >= 0 else z - 146096) // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + 3 if mp < 10 else mp - 9
    return y + (m <= 2), m, d


def binned_time_host(period, ms):
    """Scalar BinnedTime.dateToBinnedTime for planning (BinnedTime.scala:198-277)."""
    p = TimePeriod.of(period)
    if ms < 0 or ms >= _epoch_ms_max(p):
        raise IllegalArgumentException("Date exceeds indexable bounds: %d" % ms)
    esec = ms // 1000
    if p == TimePeriod.Day:
        b = ms // 86400000
        return b, ms - b * 86400000
    if p == TimePeriod.Week:
        b = ms // 604800000
        return b, esec - b * 604800
    y, m, _ = _civil_from_days(ms // 86400000)
    if p == TimePeriod.Month:
        return (y - 1970) * 12 + m - 1, esec - _days_from_civil(y, m, 1) * 86400
    return y - 1970, (esec - _days_from_civil(y, 1, 1) * 86400) // 60


@dataclass
class Z3IndexValues:
    """Z3IndexValues(sfc, geometries, spatialBounds, intervals, temporalBounds, temporalUnbounded)."""
    sfc: object
    spatialBounds: list
    intervals: list
    temporalBounds: dict = field(default_factory=dict)
    temporalUnbounded: list = field(default_factory=list)
    disjoint: bool = False


@dataclass
class Z2IndexValues:
    sfc: object
    spatialBounds: list
    disjoint: bool = False


def _clip_world(b):
    xmin, ymin, xmax, ymax = (float(v) for v in b)
    x0, y0, x1, y1 = max(xmin, -180.0), max(ymin, -90.0), min(xmax, 180.0), min(ymax, 90.0)
    if x0 > x1 or y0 > y1:
        return None
    return (x0, y0, x1, y1)


class Z3IndexKeySpace:
    """Z3 index key space for a point geometry + date attribute, no sharding by default."""

    def __init__(self, period=TimePeriod.Week, shards=0, sfc=None):
        self.period = TimePeriod.of(period)
        self.sfc = Z3SFC(self.period) if sfc is None else sfc
        self.shards = shards

    # getIndexValues (Z3IndexKeySpace.scala:97-159) for bbox + temporal predicates
    def get_index_values(self, bboxes=None, intervals=None):
        geoms = [WHOLE_WORLD] if not bboxes else bboxes
        xy = [c for c in (_clip_world(b) for b in geoms) if c is not None]
        ivs = [extract_interval(b, True) for b in (intervals or [])]
        if not xy:
            return Z3IndexValues(self.sfc, [], ivs, {}, [], disjoint=True)
        min_time, max_time = int(self.sfc.time.min), int(self.sfc.time.max)
        max_dt = _epoch_ms_max(self.period) - 1
        times = {}
        unbounded = []
        for iv in ivs:
            lo = 0 if iv.lower is None else min(max(iv.lower, 0), max_dt)       # boundsToIndexableDates
            hi = max_dt if iv.upper is None else min(max(iv.upper, 0), max_dt)
            lb, lt = binned_time_host(self.period, lo)
            ub, ut = binned_time_host(self.period, hi)
            if iv.is_bounded_both_sides:
                if lb == ub:
                    times.setdefault(lb, []).append((lt, ut))
                else:
                    times.setdefault(lb, []).append((lt, max_time))
                    times.setdefault(ub, []).append((min_time, ut))
                    for b in range(lb + 1, ub):
                        times[b] = list(self.sfc.wholePeriod)
            elif iv.lower is not None:
                times.setdefault(lb, []).append((lt, max_time))
                unbounded.append((lb + 1, SHORT_MAX))
            elif iv.upper is not None:
                times.setdefault(ub, []).append((min_time, ut))
                unbounded.append((0, ub - 1))
        return Z3IndexValues(self.sfc, xy, ivs, times, unbounded)

    def bin_ranges(self, values):
        """The epochs getRanges scans (Z3IndexKeySpace.scala:161-194), as inclusive (lo, hi) pairs."""
        if values.disjoint:
            return None
        if not values.temporalBounds and not values.temporalUnbounded:
            return []  # UnboundedRange: every bin
        out = [(b, b) for b in sorted(values.temporalBounds)]
        out += [(lo, hi) for (lo, hi) in values.temporalUnbounded]
        return out

    # getRanges (Z3IndexKeySpace.scala:161-194)
    def get_ranges(self, values, multiplier=1, target=2000):
        if values.disjoint:
            return []
        if not values.temporalBounds and not values.temporalUnbounded:
            return [("unbounded", None, None)]
        tb = values.temporalBounds
        t = max(1, (target if not tb else target // len(tb)) // multiplier)
        bins = sorted(tb)
        queries = [(values.spatialBounds, tb[b]) for b in bins]
        rs = self.sfc.ranges_batch(queries, 64, t) if queries else []
        out = []
        for b, rr in zip(bins, rs):
            out.extend(("bounded", (b, r.lower), (b, r.upper)) for r in rr)
        for (lo, hi) in values.temporalUnbounded:
            if lo == 0 and hi == SHORT_MAX:
                out.append(("unbounded", (0, 0), None))
            elif hi == SHORT_MAX:
                out.append(("lower", (lo, 0), None))
            elif lo == 0:
                out.append(("upper", None, (hi, 2**63 - 1)))
        return out

    # toIndexKey (Z3IndexKeySpace.scala:63-95), batch: row keys as an (n, 10 [+1]) uint8 array
    def to_index_keys(self, x, y, t_ms, lenient=False, shard=None):
        bins, z = self.sfc.index_keys(x, y, t_ms, lenient=lenient)
        return bins, z

    @staticmethod
    def key_bytes(bins, z, shard=None):
        """[shard?][bin BE16][z BE64] (ByteArrays.writeShort/writeLong, ByteArrays.scala:51,90-99)."""
        bins = np.asarray(bins, np.int16)
        z = np.asarray(z, np.int64)
        n = len(z)
        off = 0 if shard is None else 1
        out = np.empty((n, 10 + off), np.uint8)
        if shard is not None:
            out[:, 0] = np.asarray(shard, np.uint8)
        out[:, off:off + 2] = bins.astype(">i2").view(np.uint8).reshape(n, 2)
        out[:, off + 2:off + 10] = z.astype(">i8").view(np.uint8).reshape(n, 8)
        return out


class Z3IndexKeySpaceV4(Z3IndexKeySpace):
    """Z3IndexV4.Z3IndexKeySpaceV4 (geomesa-index-api/.../index/z3/legacy/Z3IndexV4.scala:44-51): the
    GeoMesa 1.3 key space, the same planning over LegacyZ3SFC(period)'s semi-normalized dimensions."""

    def __init__(self, period=TimePeriod.Week, shards=0):
        super().__init__(period, shards, sfc=LegacyZ3SFC(period))


class Z2IndexKeySpace:
    """Z2 index key space (geomesa-index-api/.../index/z2/Z2IndexKeySpace.scala)."""

    def __init__(self):
        self.sfc = Z2SFC()

    def get_index_values(self, bboxes=None):
        geoms = [WHOLE_WORLD] if not bboxes else bboxes
        xy = [c for c in (_clip_world(b) for b in geoms) if c is not None]
        return Z2IndexValues(self.sfc, xy, disjoint=not xy)

    # getRanges (Z2IndexKeySpace.scala:99-108): sfc.ranges(xy, 64, target) as BoundedRanges (no bin: 0)
    def get_ranges(self, values, multiplier=1, target=2000):
        if values.disjoint:
            return []
        rs = self.sfc.ranges(values.spatialBounds, 64, max(1, target // multiplier))
        return [("bounded", (0, r.lower), (0, r.upper)) for r in rs]


@dataclass
class XZ3IndexValues:
    """XZ3IndexValues(sfc, geometries, spatialBounds, intervals, temporalBounds, temporalUnbounded)."""
    sfc: object
    spatialBounds: list
    intervals: list
    temporalBounds: dict = field(default_factory=dict)
    temporalUnbounded: list = field(default_factory=list)
    disjoint: bool = False


class XZ2IndexKeySpace:
    """XZ2 index key space (geomesa-index-api/.../index/z2/XZ2IndexKeySpace.scala:28-126): the key is
    [shard][XZ2 BE64] of the geometry's envelope; every query applies the full filter (:122-125)."""

    def __init__(self, g=12):
        self.sfc = XZ2SFC(g)

    # getIndexValues (:78-95): the query geometries' bounds (a bbox is its own bounds), whole world if none
    def get_index_values(self, bboxes=None):
        geoms = [WHOLE_WORLD] if not bboxes else bboxes
        xy = [c for c in (_clip_world(b) for b in geoms) if c is not None]
        return Z2IndexValues(self.sfc, xy, disjoint=not xy)

    # getRanges (:97-102): sfc.ranges(xy, target) as BoundedRanges (bin 0 in the gm_key_range rows)
    def get_ranges(self, values, multiplier=1, target=2000):
        if values.disjoint:
            return []
        rs = self.sfc.ranges(values.spatialBounds, max(1, target // multiplier))
        return [("bounded", (0, r.lower), (0, r.upper)) for r in rs]


class XZ3IndexKeySpace:
    """XZ3 index key space (geomesa-index-api/.../index/z3/XZ3IndexKeySpace.scala:32-251): the key is
    [shard][bin BE16][XZ3 BE64] of the envelope at the dtg's period offset; every query applies the full
    filter (:247-250)."""

    def __init__(self, period=TimePeriod.Week, g=12):
        self.period = TimePeriod.of(period)
        self.sfc = XZ3SFC(g, self.period)

    # getIndexValues (:98-166)
    def get_index_values(self, bboxes=None, intervals=None):
        geoms = [WHOLE_WORLD] if not bboxes else bboxes
        xy = [c for c in (_clip_world(b) for b in geoms) if c is not None]
        ivs = [extract_interval(b, True) for b in (intervals or [])]
        if any(iv.is_bounded_both_sides and iv.lower > iv.upper for iv in ivs):   # disjoint dates (:117-120)
            return XZ3IndexValues(self.sfc, xy, ivs, {}, [], disjoint=True)
        zmin, zmax = self.sfc.zBounds
        max_dt = _epoch_ms_max(self.period) - 1
        times = {}
        unbounded = []

        def update(b, lt, ut):   # updateTime (:133-139)
            if b in times:
                times[b] = (min(times[b][0], lt), max(times[b][1], ut))
            else:
                times[b] = (lt, ut)
        for iv in ivs:
            lo = 0 if iv.lower is None else min(max(iv.lower, 0), max_dt)       # boundsToIndexableDates
            hi = max_dt if iv.upper is None else min(max(iv.upper, 0), max_dt)
            lb, lt = binned_time_host(self.period, lo)
            ub, ut = binned_time_host(self.period, hi)
            if iv.is_bounded_both_sides:
                if lb == ub:
                    update(lb, float(lt), float(ut))
                else:
                    update(lb, float(lt), zmax)
                    update(ub, zmin, float(ut))
                    for b in range(lb + 1, ub):
                        times[b] = (zmin, zmax)
            elif iv.lower is not None:
                update(lb, float(lt), zmax)
                unbounded.append((lb + 1, SHORT_MAX))
            elif iv.upper is not None:
                update(ub, zmin, float(ut))
                unbounded.append((0, ub - 1))
        return XZ3IndexValues(self.sfc, xy, ivs, times, unbounded, disjoint=not xy)

    # getRanges (:168-201): per bin the XZ3 ranges of the boxes x the bin's times, target split over bins
    def get_ranges(self, values, multiplier=1, target=2000):
        if values.disjoint:
            return []
        tb, ub = values.temporalBounds, values.temporalUnbounded
        if not tb and not ub:
            return [("unbounded", None, None)]
        t = max(1, (target if not tb else target // len(tb)) // multiplier)
        bins = sorted(tb)
        queries = [[(x0, y0, tb[b][0], x1, y1, tb[b][1]) for (x0, y0, x1, y1) in values.spatialBounds] for b in bins]
        rs = self.sfc.ranges_batch(queries, t) if queries else []
        out = []
        for b, rr in zip(bins, rs):
            out.extend(("bounded", (b, r.lower), (b, r.upper)) for r in rr)
        for (lo, hi) in ub:
            if hi == SHORT_MAX:
                out.append(("lower", (lo, 0), None))
            elif lo == 0:
                out.append(("upper", None, (hi, 2**63 - 1)))
            else:
                out.append(("unbounded", (0, 0), None))
        return out
