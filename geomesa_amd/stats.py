"""Z3Histogram: the statistics caller of the Z3 curve.

Mirrors geomesa-utils/src/main/scala/org/locationtech/geomesa/utils/stats/Z3Histogram.scala
(observe / unobserve :101-128, toKey :80-86, count / directIndex / indexOf :63-72, +=  :145-160,
isEmpty / clear :169-171, splitByTime :95-99, toJsonObject :163-167) over batches of point features:
the per-feature work (BinnedTime + Z3SFC.index + LongBinning.directIndex + the increment) runs in
the gm_z3_histogram kernel; this class keeps the binMap as a dense device block of int64 counters
for a window of time bins [bin_lo, bin_lo + n_bins) plus a per-bin "present" flag (the map's key
set), and widens the window when a batch has features outside it.
"""
import numpy as np

from . import _lib
from ._lib import check, ptr
from .curve import BinnedTime, TimePeriod, Z3SFC, _dev_col, _torch

_JSON_FMT = {TimePeriod.Day: "%05d", TimePeriod.Week: "%04d", TimePeriod.Month: "%03d", TimePeriod.Year: "%02d"}
_PERIOD_NAME = {TimePeriod.Day: "day", TimePeriod.Week: "week", TimePeriod.Month: "month", TimePeriod.Year: "year"}
MIN_Z, MAX_Z = 0, (1 << 63) - 1  # Z3Histogram.scala:53-54 for every period (see gm_stats.hip)


def long_binning_index(value, length, lo=MIN_Z, hi=MAX_Z):
    """LongBinning.directIndex (BinnedArray.scala:185-201), scalar host form."""
    if value < lo or value > hi:
        return -1
    bs = float(hi - lo) / length
    i = int(np.floor(float(value - lo) / bs))
    if i < 0 or i > length:
        return -1
    return length - 1 if i == length else i


class Z3Histogram:
    """Stat.Z3Histogram(geom, dtg, period, length) over point columns (x, y, epoch-ms t)."""

    def __init__(self, geom="geom", dtg="dtg", period=TimePeriod.Week, length=1024, device=None):
        self.geom, self.dtg, self.length = geom, dtg, int(length)
        self.period = TimePeriod.of(period)
        self.sfc = Z3SFC(self.period)
        self._device = device
        self.bin_lo = None
        self.n_bins = 0
        self.counts = None    # int64 [n_bins, length] on the device
        self.present = None   # uint8 [n_bins]
        self.skipped = 0      # features whose toKey threw (the Scala code logs a warning per feature)

    # ------------------------------------------------------------------ window management
    def _alloc(self, lo, n):
        torch = _torch()
        dev = torch.device("cuda", _lib.context(self._device).device)
        counts = torch.zeros((n, self.length), dtype=torch.int64, device=dev)
        present = torch.zeros(n, dtype=torch.uint8, device=dev)
        if self.counts is not None:
            off = self.bin_lo - lo
            counts[off:off + self.n_bins] = self.counts
            present[off:off + self.n_bins] = self.present
        self.bin_lo, self.n_bins, self.counts, self.present = lo, n, counts, present

    def _cover(self, t):
        """Widen the window to the valid time bins of batch t (BinnedTime per feature, invalid ones ignored)."""
        b, _, s = BinnedTime.time_to_binned_time(self.period, t, status=True)
        ok = s == 0
        if not bool(ok.any()):
            return
        lo, hi = int(b[ok].min()), int(b[ok].max())
        if self.counts is not None:
            lo, hi = min(lo, self.bin_lo), max(hi, self.bin_lo + self.n_bins - 1)
            if lo == self.bin_lo and hi == self.bin_lo + self.n_bins - 1:
                return
        self._alloc(lo, hi - lo + 1)

    def _run(self, x, y, t, unobserve, counts, present, tally):
        ctx = _lib.context(self._device)
        n = x.numel()
        check(ctx.lib.gm_z3_histogram(ctx.handle, ptr(x), ptr(y), ptr(t), n, self.period, self.length,
                                      int(unobserve), self.bin_lo, self.n_bins, ptr(present), ptr(counts),
                                      ptr(tally)), "gm_z3_histogram")

    def _apply(self, x, y, t_ms, unobserve):
        torch = _torch()
        x = _dev_col(x, torch.float64); y = _dev_col(y, torch.float64); t = _dev_col(t_ms, torch.int64)
        if x.numel() == 0:
            return
        if self.counts is None:
            if unobserve:
                return  # binMap is empty: nothing to take away
            self._cover(t)
            if self.counts is None:  # every feature failed BinnedTime
                self.skipped += x.numel()
                return
        tally = torch.zeros(2, dtype=torch.int64, device=x.device)
        if unobserve:
            # bins outside the window are absent from binMap: unobserve ignores them
            self._run(x, y, t, True, self.counts, self.present, tally)
            self.skipped += int(tally[0])
            return
        # straight into the binMap block: features of bins outside the window are left out and
        # counted in tally[1] (no per-batch scratch block)
        self._run(x, y, t, False, self.counts, self.present, tally)
        self.skipped += int(tally[0])
        if int(tally[1]) > 0:
            # widen to the batch's bins, then add only the features of the new rows: the rows below
            # and above the old window are contiguous row blocks of the dense counts
            lo0, hi0 = self.bin_lo, self.bin_lo + self.n_bins   # [lo0, hi0)
            self._cover(t)
            extra = torch.zeros(2, dtype=torch.int64, device=x.device)
            below, above = lo0 - self.bin_lo, self.bin_lo + self.n_bins - hi0
            if below > 0:
                self._run_rows(x, y, t, self.bin_lo, 0, below, extra)
            if above > 0:
                self._run_rows(x, y, t, hi0, hi0 - self.bin_lo, above, extra)

    def _run_rows(self, x, y, t, bin_lo, row0, rows, tally):
        ctx = _lib.context(self._device)
        check(ctx.lib.gm_z3_histogram(ctx.handle, ptr(x), ptr(y), ptr(t), x.numel(), self.period, self.length, 0,
                                      bin_lo, rows, ptr(self.present[row0:row0 + rows]),
                                      ptr(self.counts[row0:row0 + rows]), ptr(tally)), "gm_z3_histogram")

    # ------------------------------------------------------------------ Stat API
    def observe(self, x, y, t_ms):
        """Z3Histogram.observe for a batch of point features (Z3Histogram.scala:101-111)."""
        self._apply(x, y, t_ms, False)

    def unobserve(self, x, y, t_ms):
        """Z3Histogram.unobserve (Z3Histogram.scala:113-123): lenient toKey, present bins only."""
        self._apply(x, y, t_ms, True)

    def time_bins(self):
        if self.present is None:
            return []
        idx = np.nonzero(self.present.cpu().numpy())[0]
        return [int(i) + self.bin_lo for i in idx]

    def _row(self, time_bin):
        if self.present is None:
            return None
        r = time_bin - self.bin_lo
        if r < 0 or r >= self.n_bins or not int(self.present[r]):
            return None
        return r

    def count(self, time_bin, i):
        r = self._row(time_bin)
        return 0 if r is None else int(self.counts[r, i])

    def bins(self, time_bin):
        """BinnedArray.counts for one time bin (host int64 array) or None when absent."""
        r = self._row(time_bin)
        return None if r is None else self.counts[r].cpu().numpy()

    def direct_index(self, time_bin, z):
        return -1 if self._row(time_bin) is None else long_binning_index(int(z), self.length)

    def index_of(self, x, y, t_ms):
        """indexOf((geom, date)) (Z3Histogram.scala:67-70): non-lenient toKey, then directIndex."""
        b, z = self.sfc.index_keys([x], [y], [t_ms])
        return int(b[0]), self.direct_index(int(b[0]), int(z[0]))

    def median_value(self, time_bin, i):
        """medianValue (Z3Histogram.scala:72, BinnedArray.scala:205-211) -> (x, y, offset in the period)."""
        bs = float(MAX_Z - MIN_Z) / self.length
        v = MIN_Z + int(np.floor(bs / 2 + bs * i + 0.5))  # math.round
        v = min(v, MAX_Z)
        x, y, t = self.sfc.invert([v])
        return float(x[0]), float(y[0]), int(t[0])

    def is_empty(self):
        return self.counts is None or not bool((self.counts != 0).any())

    def clear(self):
        if self.counts is not None:
            self.counts.zero_()

    def __iadd__(self, other):
        """+= (Z3Histogram.scala:145-160): counts of shared bins add, new bins are copied in."""
        if self.length != other.length:
            raise NotImplementedError("Can only add z3 histograms with the same length")
        if other.counts is None:
            return self
        if self.counts is None:
            self._alloc(other.bin_lo, other.n_bins)
        lo = min(self.bin_lo, other.bin_lo)
        hi = max(self.bin_lo + self.n_bins, other.bin_lo + other.n_bins)
        if lo != self.bin_lo or hi != self.bin_lo + self.n_bins:
            self._alloc(lo, hi - lo)
        off = other.bin_lo - self.bin_lo
        self.counts[off:off + other.n_bins] += other.counts * other.present.unsqueeze(1).to(other.counts.dtype)
        self.present[off:off + other.n_bins] |= other.present
        return self

    def __add__(self, other):
        out = Z3Histogram(self.geom, self.dtg, self.period, self.length, self._device)
        out += self
        out += other
        return out

    def all_reduce(self, pg):
        """Merge this rank's histogram with every other rank's (`+=` over the process group, RCCL).
        The merged block comes back on this histogram's device whatever the backend's transport
        device (gloo reduces on the CPU)."""
        from .shard import merge_histograms
        c, p, lo = merge_histograms(pg, self.counts, self.present, self.bin_lo, self.length)
        if c is not None:
            torch = _torch()
            dev = torch.device("cuda", _lib.context(self._device).device)
            self.counts, self.present = c.to(dev).contiguous(), p.to(dev).contiguous()
            self.bin_lo, self.n_bins = lo, c.shape[0]
        return self

    def split_by_time(self):
        out = []
        for b in self.time_bins():
            h = Z3Histogram(self.geom, self.dtg, self.period, self.length, self._device)
            h._alloc(b, 1)
            h.counts[0] = self.counts[b - self.bin_lo]
            h.present[0] = 1
            out.append((b, h))
        return out

    def to_json_object(self):
        """toJsonObject (Z3Histogram.scala:163-167)."""
        name, fmt = _PERIOD_NAME[self.period], _JSON_FMT[self.period]
        return [{("%s-" + fmt) % (name, b): {"bins": [int(c) for c in self.bins(b)]}} for b in self.time_bins()]

    def is_equivalent(self, other):
        if not (self.period == other.period and self.length == other.length):
            return False
        if self.time_bins() != other.time_bins():
            return False
        return all(np.array_equal(self.bins(b), other.bins(b)) for b in self.time_bins())


__all__ = ["Z3Histogram", "long_binning_index", "MIN_Z", "MAX_Z"]
