"""GPU parity of gm_z3_histogram (Z3Histogram observe / unobserve) against the C oracle; bit-exact counts."""
import datetime

import numpy as np
import pytest

from test_gpu_parity import T2020, T2021, edge_points, random_points

pytestmark = pytest.mark.gpu
WEEK = 1


def _dev(a, torch):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def run_hist(x, y, t, period, length, lo, nb, unobserve=False, present=None, counts=None):
    import torch
    from geomesa_amd import _lib
    ctx = _lib.context()
    X, Y, T = _dev(x, torch), _dev(y, torch), _dev(t, torch)
    P = _dev(present if present is not None else np.zeros(nb, np.uint8), torch)
    C = _dev(counts if counts is not None else np.zeros((nb, length), np.int64), torch)
    tally = torch.zeros(2, dtype=torch.int64, device="cuda")
    _lib.check(ctx.lib.gm_z3_histogram(ctx.handle, _lib.ptr(X), _lib.ptr(Y), _lib.ptr(T), len(x), period, length,
                                       int(unobserve), lo, nb, _lib.ptr(P), _lib.ptr(C), _lib.ptr(tally)),
               "gm_z3_histogram")
    torch.cuda.synchronize()
    return P.cpu().numpy(), C.cpu().numpy(), tally.cpu().numpy()


def inputs(n):
    x, y, t = random_points(n)
    ex, ey, et = edge_points()
    return np.concatenate([x, ex]), np.concatenate([y, ey]), np.concatenate([t, et])


# LDS-private path (n_bins * length + n_bins <= 32768) and the global-atomic path
@pytest.mark.parametrize("period,length,lo,nb", [
    (WEEK, 512, 2600, 53), (WEEK, 1024, 2600, 53), (WEEK, 4096, 2600, 53), (WEEK, 64, 2590, 70), (0, 128, 18260, 200),
    (2, 1000, 595, 14), (3, 10000, 48, 4), (WEEK, 1, 0, 1)])
def test_z3_histogram_parity(gpu, oracle, period, length, lo, nb):
    x, y, t = inputs(300_001)
    P, C, tl = run_hist(x, y, t, period, length, lo, nb)
    op, oc, ot = oracle.z3_histogram(x, y, t, length, lo, nb, period=period)
    assert np.array_equal(tl, ot)
    assert np.array_equal(P, op)
    assert np.array_equal(C, oc)
    # unobserve half the features on top (lenient toKey, present bins only), accumulating
    h = len(x) // 2
    P2, C2, tl2 = run_hist(x[:h], y[:h], t[:h], period, length, lo, nb, True, P, C)
    oracle.z3_histogram(x[:h], y[:h], t[:h], length, lo, nb, unobserve=True, period=period, present=op, counts=oc,
                        tally=ot)
    assert np.array_equal(C2, oc)
    assert np.array_equal(P2, op)


def _points_with_normalized(oracle, xn, yn, tn, week_bin=2610):
    """Points whose normalized (lon, lat, week offset) are exactly (xn, yn, tn) where reachable: cell
    centres for x / y; for t the second whose normalized offset is tn (skipped when none is)."""
    xs, ys, ts = [], [], []
    for a, b, c in zip(xn, yn, tn):
        x = -180.0 + (a + 0.5) * (360.0 / 2 ** 21)
        y = -90.0 + (b + 0.5) * (180.0 / 2 ** 21)
        assert oracle.normalize(-180.0, 180.0, 21, x) == a and oracle.normalize(-90.0, 90.0, 21, y) == b
        # a normalized week offset advances ~3.5 per second: not every value is reachable, so the
        # lowest 3 bits of tn (z bits 2, 5, 8: below any carry) are lowered until one is
        done = False
        for cj in range(c, max(c - 8, -1), -1):
            sec = int(cj * 604800 / 2 ** 21)
            for s_ in range(sec - 2, sec + 4):
                if 0 <= s_ < 604800 and oracle.normalize(0.0, 604800.0, 21, float(s_)) == cj:
                    xs.append(x); ys.append(y); ts.append(week_bin * 604800000 + s_ * 1000 + 7)
                    done = True
                    break
            if done:
                break
    return np.array(xs), np.array(ys), np.array(ts, np.int64)


@pytest.mark.parametrize("length", [512, 1024, 2048, 64])
def test_z3_histogram_top_bits_rounding(gpu, oracle, length):
    """Power-of-two lengths bin from the top bits of z (gm_stats.hip TOP path) unless the Long -> Double
    rounding of directIndex can carry into them: keys whose bits below a bin boundary are all ones
    (the rounding carries into the next bin), one zero bit at every position below the boundary (no
    carry), and random keys, against the oracle's exact directIndex."""
    m = length.bit_length() - 1
    s_ = (63 - m) // 3
    rng = np.random.default_rng(length)
    xn, yn, tn = [], [], []
    for k in range(1, 1 << (21 - s_)):
        top = k << s_
        for dims in range(3):   # all ones below the boundary, in every dim (a carry) ...
            xn.append(top - 1); yn.append(top - 1); tn.append(top - 1)
            for zb in range(3, s_):   # ... and with one zero bit in one dim (no carry past it)
                v = [top - 1] * 3
                v[dims] &= ~(1 << zb)
                xn.append(v[0]); yn.append(v[1]); tn.append(v[2])
    r = rng.integers(0, 2 ** 21, (3, 4000))
    xn += r[0].tolist(); yn += r[1].tolist(); tn += r[2].tolist()
    x, y, t = _points_with_normalized(oracle, xn, yn, tn)
    assert len(x) > 200
    lo, nb = 2609, 3
    P, C, tl = run_hist(x, y, t, WEEK, length, lo, nb)
    op, oc, ot = oracle.z3_histogram(x, y, t, length, lo, nb, period=WEEK)
    assert np.array_equal(C, oc) and np.array_equal(P, op) and np.array_equal(tl, ot)


@pytest.mark.parametrize("length,lo,nb", [(1024, 2600, 53), (64, 2607, 4)])
def test_z3_histogram_hot_counters(gpu, oracle, length, lo, nb):
    """8M features on 3 positions: tens of thousands of increments per counter per workgroup, past the
    int32 path and the packed 21-bit counters (length 1024 x 53 runs the WIDE path)."""
    rng = np.random.default_rng(9)
    n = 8_000_000
    k = rng.integers(0, 3, n)
    x = np.array([10.0, -75.5, 139.7])[k]
    y = np.array([47.0, 40.1, 35.6])[k]
    t = np.array([T2020 + 5 * 86400000, T2020 + 5 * 86400000 + 1, T2020 + 9 * 86400000])[k]
    P, C, tl = run_hist(x, y, t, WEEK, length, lo, nb)
    op, oc, ot = oracle.z3_histogram(x, y, t, length, lo, nb, period=WEEK)
    assert np.array_equal(C, oc) and np.array_equal(P, op) and np.array_equal(tl, ot)
    assert C.max() > 2_000_000
    h = 6_000_000
    P2, C2, _ = run_hist(x[:h], y[:h], t[:h], WEEK, length, lo, nb, True, P, C)
    oracle.z3_histogram(x[:h], y[:h], t[:h], length, lo, nb, unobserve=True, period=WEEK, present=op, counts=oc,
                        tally=ot)
    assert np.array_equal(C2, oc) and np.array_equal(P2, op)


@pytest.mark.parametrize("grid,length,nb,aligned", [(1, 1024, 53, True), (3, 1024, 53, True), (1, 2048, 54, True),
                                                     (1, 1024, 53, False)])
def test_z3_histogram_wide_counter_drains(gpu, oracle, grid, length, nb, aligned):
    """The packed 21-bit LDS counters (WIDE: histograms past int32 LDS) drain to the device counters on a
    fixed schedule so no field carries into its neighbour: with one or three workgroups
    (GM_PARAM_HIST_GRID) every workgroup counts millions of features into three hot counters -- past
    2^21 per field -- and drains many times; observe, then unobserve (fields biased at 2^20, drained
    twice as often) of 6M of them, bit-exact against the oracle.  length 2048 x 54 takes two LDS passes;
    an unaligned column takes the scalar loop."""
    import torch
    from geomesa_amd import _lib
    rng = np.random.default_rng(12)
    n = 8_000_001
    k = rng.integers(0, 3, n)
    x = np.array([10.0, -75.5, 139.7])[k]
    y = np.array([47.0, 40.1, 35.6])[k]
    t = np.array([T2020 + 5 * 86400000, T2020 + 5 * 86400000 + 1, T2020 + 9 * 86400000])[k]
    if not aligned:   # an odd element in front: the columns' data start 8 B off the 16-B grid
        x, y, t = (np.concatenate([v[:1], v]) for v in (x, y, t))
    ctx = _lib.context()
    ctx.set_param(_lib.GM_PARAM_HIST_GRID, grid)
    try:
        lo = 2600
        sl = slice(1, None) if not aligned else slice(None)

        def run(xs, ys, ts, unobs=False, P0=None, C0=None):
            X, Y, T = (_dev(v, torch) for v in (xs, ys, ts))
            if not aligned:
                X, Y, T = X[1:], Y[1:], T[1:]
            P = _dev(P0 if P0 is not None else np.zeros(nb, np.uint8), torch)
            C = _dev(C0 if C0 is not None else np.zeros((nb, length), np.int64), torch)
            tl = torch.zeros(2, dtype=torch.int64, device="cuda")
            _lib.check(ctx.lib.gm_z3_histogram(ctx.handle, _lib.ptr(X), _lib.ptr(Y), _lib.ptr(T), X.numel(), WEEK, length,
                                               int(unobs), lo, nb, _lib.ptr(P), _lib.ptr(C), _lib.ptr(tl)), "hist")
            return P.cpu().numpy(), C.cpu().numpy(), tl.cpu().numpy()
        P, C, tl = run(x, y, t)
        op, oc, ot = oracle.z3_histogram(x[sl], y[sl], t[sl], length, lo, nb, period=WEEK)
        assert np.array_equal(C, oc) and np.array_equal(P, op) and np.array_equal(tl, ot)
        assert C.max() > (1 << 21)          # a field's worth, several times over, through one workgroup's drains
        h = 6_000_000 + (0 if aligned else 1)
        P2, C2, _ = run(x[:h], y[:h], t[:h], True, P, C)
        oracle.z3_histogram(x[sl][:6_000_000], y[sl][:6_000_000], t[sl][:6_000_000], length, lo, nb, unobserve=True,
                            period=WEEK, present=op, counts=oc, tally=ot)
        assert np.array_equal(C2, oc) and np.array_equal(P2, op)
    finally:
        ctx.set_param(_lib.GM_PARAM_HIST_GRID, 0)


def test_z3_histogram_unaligned_and_small(gpu, oracle):
    import torch
    from geomesa_amd import _lib
    x, y, t = inputs(10_001)
    for off, n in [(1, 5001), (3, 1), (0, 2), (1, 0)]:
        xs, ys, ts = x[off:off + n], y[off:off + n], t[off:off + n]
        X = _dev(x, torch)[off:off + n]; Y = _dev(y, torch)[off:off + n]; T = _dev(t, torch)[off:off + n]
        P = torch.zeros(53, dtype=torch.uint8, device="cuda")
        C = torch.zeros((53, 256), dtype=torch.int64, device="cuda")
        tl = torch.zeros(2, dtype=torch.int64, device="cuda")
        ctx = _lib.context()
        _lib.check(ctx.lib.gm_z3_histogram(ctx.handle, _lib.ptr(X), _lib.ptr(Y), _lib.ptr(T), n, WEEK, 256, 0, 2600,
                                           53, _lib.ptr(P), _lib.ptr(C), _lib.ptr(tl)), "gm_z3_histogram")
        op, oc, ot = oracle.z3_histogram(xs, ys, ts, 256, 2600, 53)
        assert np.array_equal(C.cpu().numpy(), oc) and np.array_equal(tl.cpu().numpy(), ot)
        assert np.array_equal(P.cpu().numpy(), op)


def test_z3_histogram_rejects_bad_args(gpu):
    import torch
    from geomesa_amd import _lib
    ctx = _lib.context()
    z = torch.zeros(4, dtype=torch.int64, device="cuda")
    for period, length, lo, nb in [(7, 16, 0, 1), (1, 0, 0, 1), (1, 16, 0, 0), (1, 16, 32767, 2), (1, 16, -32769, 1)]:
        rc = ctx.lib.gm_z3_histogram(ctx.handle, _lib.ptr(z), _lib.ptr(z), _lib.ptr(z), 1, period, length, 0, lo, nb,
                                     _lib.ptr(z), _lib.ptr(z), _lib.ptr(z))
        assert rc == _lib.GM_E_INVALID


def ms(s):
    return int(datetime.datetime.fromisoformat(s + "+00:00").timestamp() * 1000)


def test_z3histogram_reference_kat(gpu):  # Z3HistogramTest.scala:45-52, 95-106 through the host mirror
    from geomesa_amd.stats import Z3Histogram
    i = np.arange(100)
    x = -i.astype(np.float64); y = (i // 2).astype(np.float64)
    t = np.array([ms("2012-01-01T%02d:00:00" % (k % 24)) for k in i], np.int64)
    h = Z3Histogram("geom", "dtg", "week", 1024)
    assert h.is_empty()
    h.observe(x, y, t)
    assert not h.is_empty()
    for k in range(100):
        w, idx = h.index_of(x[k], y[k], int(t[k]))
        assert 1 <= h.count(w, idx) <= 21
    # serialize-style equivalence: toJson of a + b equals the counts doubled
    h2 = h + h
    (label, body), = h2.to_json_object()[0].items()
    assert label.startswith("week-") and sum(body["bins"]) == 200
    h.clear()
    assert h.is_empty()
    for k in range(100):
        w, idx = h.index_of(x[k], y[k], int(t[k]))
        assert h.count(w, idx) == 0


def test_z3histogram_window_grows(gpu, oracle):
    from geomesa_amd.stats import Z3Histogram
    x, y, t = random_points(50_000)
    wk = 604800000
    h = Z3Histogram(period="week", length=256)
    h.observe(x[:25_000], y[:25_000], t[:25_000])
    t2 = t[25_000:] + 30 * wk            # later weeks: the window must widen
    h.observe(x[25_000:], y[25_000:], t2)
    tt = np.concatenate([t[:25_000], t2])
    lo, nb = h.bin_lo, h.n_bins
    op, oc, ot = oracle.z3_histogram(x, y, tt, 256, lo, nb)
    assert ot.tolist() == [0, 0]
    assert np.array_equal(h.counts.cpu().numpy(), oc)
    assert np.array_equal(h.present.cpu().numpy(), op)
    parts = h.split_by_time()
    assert sum(int(p.counts.sum()) for _, p in parts) == 50_000
    assert T2020 < T2021


def test_z3histogram_window_grows_both_sides(gpu, oracle):
    """A batch with features below, inside and above the window: the in-window features go straight
    into the binMap block, the others into the rows the window gains on each side."""
    from geomesa_amd.stats import Z3Histogram
    x, y, t = random_points(60_000)
    wk = 604800000
    h = Z3Histogram(period="week", length=128)
    h.observe(x[:20_000], y[:20_000], t[:20_000] + 20 * wk)
    t2 = t[20_000:].copy()
    t2[::3] += 45 * wk                     # above the window
    t2[1::3] += 20 * wk                    # inside
    h.observe(x[20_000:], y[20_000:], t2)  # the rest below it
    tt = np.concatenate([t[:20_000] + 20 * wk, t2])
    op, oc, ot = oracle.z3_histogram(x, y, tt, 128, h.bin_lo, h.n_bins)
    assert ot.tolist() == [0, 0] and h.skipped == 0
    assert np.array_equal(h.counts.cpu().numpy(), oc) and np.array_equal(h.present.cpu().numpy(), op)


def test_z3histogram_all_reduce_then_observe(gpu, oracle):
    """all_reduce over a gloo group (CPU transport) hands the merged block back on the
    histogram's device, so the next observe runs on device memory."""
    import os
    import socket
    import torch.distributed as dist
    from geomesa_amd.stats import Z3Histogram
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        x, y, t = random_points(40_000)
        h = Z3Histogram(period="week", length=64)
        h.observe(x[:20_000], y[:20_000], t[:20_000])
        h.all_reduce(dist)
        assert h.counts.is_cuda and h.present.is_cuda
        h.observe(x[20_000:], y[20_000:], t[20_000:])
        op, oc, ot = oracle.z3_histogram(x, y, t, 64, h.bin_lo, h.n_bins)
        assert np.array_equal(h.counts.cpu().numpy(), oc) and np.array_equal(h.present.cpu().numpy(), op)
    finally:
        dist.destroy_process_group()
