"""Z3Histogram: the C oracle (gmo_z3_histogram) pinned to the reference's own Z3HistogramTest, plus the
host-side LongBinning index.  CPU only.

Fixtures: geomesa-utils/src/test/scala/org/locationtech/geomesa/utils/stats/Z3HistogramTest.scala
(features from StatTestHelper.scala:18-21: POINT(-i i/2) at 2012-01-01T{i%24}:00:00Z, i = 0..99).
"""
import datetime

import numpy as np

WEEK = 1
MAXZ = (1 << 63) - 1


def ms(s):
    return int(datetime.datetime.fromisoformat(s + "+00:00").timestamp() * 1000)


def stat_features():  # StatTestHelper.scala:18-21
    i = np.arange(100)
    x = -i.astype(np.float64)
    y = (i // 2).astype(np.float64)
    t = np.array([ms("2012-01-01T%02d:00:00" % (k % 24)) for k in i], np.int64)
    return x, y, t


def observe(oracle, length=1024):
    x, y, t = stat_features()
    b, _, _ = oracle.z3_index_key_batch(x, y, t, period=WEEK)
    lo = int(b.min())
    pres, counts, tally = oracle.z3_histogram(x, y, t, length, lo, 1)
    return lo, pres, counts, tally


def test_z3histogram_correctly_bins(oracle):  # Z3HistogramTest.scala:44-51
    lo, pres, counts, tally = observe(oracle)
    assert tally.tolist() == [0, 0] and pres.tolist() == [1]
    assert counts.sum() == 100
    x, y, t = stat_features()
    b, z, st = oracle.z3_index_key_batch(x, y, t, period=WEEK)
    for k in range(100):
        assert b[k] == lo
        idx = oracle.long_binning_index(0, MAXZ, 1024, int(z[k]))
        assert 1 <= counts[0, idx] <= 21


def test_z3histogram_clear_and_unobserve(oracle):  # Z3HistogramTest.scala:95-106 ("clear")
    lo, pres, counts, tally = observe(oracle)
    x, y, t = stat_features()
    oracle.z3_histogram(x, y, t, 1024, lo, 1, unobserve=True, present=pres, counts=counts, tally=tally)
    assert not counts.any()          # isEmpty after taking every feature away
    # POINT(-180 -90) at 2012-01-01 falls in the same week, in a counter that now holds nothing
    b, z, _ = oracle.z3_index_key_batch([-180.0], [-90.0], [ms("2012-01-01T00:00:00")], period=WEEK)
    assert b[0] == lo and counts[0, oracle.long_binning_index(0, MAXZ, 1024, int(z[0]))] == 0


def test_z3histogram_skips_and_window(oracle):
    # toKey failures (out-of-bounds lon, pre-1970 time) are skipped; a bin outside the window is tallied
    wk = 604800000
    x = np.array([0.0, 200.0, 0.0, 0.0]); y = np.zeros(4); t = np.array([5 * wk, 5 * wk, -1, 9 * wk], np.int64)
    pres, counts, tally = oracle.z3_histogram(x, y, t, 16, 5, 2)
    assert tally.tolist() == [2, 1] and pres.tolist() == [1, 0] and counts.sum() == 1
    # unobserve is lenient (200 clamps to 180) and only touches present bins
    oracle.z3_histogram(x, y, t, 16, 5, 2, unobserve=True, present=pres, counts=counts, tally=tally)
    assert counts.sum() == -1 and tally.tolist() == [3, 2]


def test_long_binning_index(oracle):  # BinnedArray.scala:195-201
    from geomesa_amd.stats import long_binning_index
    rng = np.random.default_rng(7)
    vals = [0, 1, MAXZ, MAXZ - 1, -1, 1 << 62, (1 << 62) - 1] + [int(v) for v in rng.integers(0, MAXZ, 200)]
    for length in (1, 7, 1024, 10000, 65536):
        bs = float(MAXZ) / length
        edges = [int(bs * k) + d for k in range(0, length, max(1, length // 8)) for d in (-1, 0, 1)]
        for v in vals + edges:
            assert long_binning_index(v, length) == oracle.long_binning_index(0, MAXZ, length, v), (v, length)
    assert oracle.long_binning_index(0, MAXZ, 1024, MAXZ) == 1023
    assert oracle.long_binning_index(0, MAXZ, 1024, -5) == -1
