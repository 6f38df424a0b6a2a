"""GPU parity: the HIP library (through the C ABI) against the C oracle on the same seeded inputs.

Integer/byte/index outputs must be bit-exact; floating outputs (invert) are compared bit-for-bit as
well (the JVM arithmetic is reproduced exactly, so no tolerance is needed).
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x67656F6D65736121
T2020, T2021 = 1577836800000, 1609459200000


def as_np(t):
    return t.detach().cpu().numpy()


def f64_bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def edge_points():
    nx = math.nextafter
    xs = [-180.0, 180.0, nx(180.0, 0), nx(-180.0, 0), 0.0, -0.0, 179.99999999999997, 180.0000001, -180.1,
          float("nan"), float("inf"), -float("inf"), 1e-300, -1e-300, 45.0, 45.000000001]
    ys = [-90.0, 90.0, nx(90.0, 0), nx(-90.0, 0), 0.0, -0.0, 89.99999999999999, 90.0000001, -90.1, float("nan"),
          float("inf"), -float("inf"), 1e-300, -1e-300, 49.0, 49.000000001]
    wk = 604800000
    ts = [0, -1, 1, wk - 1, wk, wk + 1, 2370 * wk + 172801000, 32768 * wk - 1, 32768 * wk, 2**62, -2**62,
          86400000 * 32768 - 1, 86400000 * 32768, T2020, T2021 - 1, 999]
    X, Y, T = np.meshgrid(np.array(xs), np.array(ys), np.array(ts, np.int64), indexing="ij")
    return X.ravel(), Y.ravel(), T.ravel()


def random_points(n, seed=SEED):
    rng = np.random.default_rng(seed & 0xFFFFFFFF)
    x = rng.uniform(-180, 180, n)
    y = rng.uniform(-90, 90, n)
    t = rng.integers(T2020, T2021, n)
    return x, y, t


@pytest.mark.parametrize("period", [0, 1, 2, 3])
@pytest.mark.parametrize("lenient", [False, True])
def test_z3_index_key_parity(gpu, oracle, period, lenient):
    from geomesa_amd.curve import Z3SFC
    x, y, t = random_points(200_003)
    ex, ey, et = edge_points()
    x = np.concatenate([x, ex]); y = np.concatenate([y, ey]); t = np.concatenate([t, et])
    sfc = Z3SFC(period)
    b, z, s = sfc.index_keys(x, y, t, lenient=lenient, status=True)
    ob, oz, os_ = oracle.z3_index_key_batch(x, y, t, lenient=lenient, period=period)
    assert np.array_equal(as_np(s), os_)
    assert np.array_equal(as_np(b), ob)
    assert np.array_equal(as_np(z), oz)


def test_z3_index_key_raises_like_jvm(gpu):
    from geomesa_amd.curve import IllegalArgumentException, Z3SFC
    with pytest.raises(IllegalArgumentException):
        Z3SFC("week").index_keys([0.0, 190.0], [0.0, 0.0], [T2020, T2020])
    with pytest.raises(IllegalArgumentException):   # BinnedTime throws even when lenient
        Z3SFC("week").index_keys([0.0], [0.0], [-5], lenient=True)


def test_z3_index_key_odd_and_unaligned(gpu, oracle):
    import torch
    from geomesa_amd.curve import Z3SFC
    x, y, t = random_points(1001)
    tx = torch.from_numpy(x).cuda(); ty = torch.from_numpy(y).cuda(); tt = torch.from_numpy(t).cuda()
    for sl in [slice(0, 1001), slice(1, 1000), slice(3, 4), slice(0, 0)]:
        b, z = Z3SFC("week").index_keys(tx[sl], ty[sl], tt[sl])
        ob, oz, _ = oracle.z3_index_key_batch(x[sl], y[sl], t[sl])
        assert np.array_equal(as_np(z), oz) and np.array_equal(as_np(b), ob)


@pytest.mark.parametrize("precision", [21, 17, 1])
@pytest.mark.parametrize("period", [1, 3])
def test_z3_index_offset_parity(gpu, oracle, period, precision):
    from geomesa_amd.curve import Z3SFC, max_offset
    rng = np.random.default_rng(7)
    n = 50_000
    x = rng.uniform(-181, 181, n); y = rng.uniform(-91, 91, n)
    t = rng.integers(-10, max_offset(period) + 10, n)
    z, s = Z3SFC(period, precision).index(x, y, t, lenient=False, status=True)
    zl = Z3SFC(period, precision).index(x, y, t, lenient=True)
    for i in range(0, n, 97):
        st, oz = oracle.z3_index(x[i], y[i], int(t[i]), False, period, precision)
        assert int(as_np(s)[i]) == st and (st or int(as_np(z)[i]) == oz)
        st, oz = oracle.z3_index(x[i], y[i], int(t[i]), True, period, precision)
        assert int(as_np(zl)[i]) == oz


@pytest.mark.parametrize("period", [0, 1, 2, 3])
def test_z3_invert_parity(gpu, oracle, period):
    from geomesa_amd.curve import Z3SFC
    rng = np.random.default_rng(11)
    z = np.concatenate([rng.integers(0, 2**63 - 1, 100_001, dtype=np.int64),
                        rng.integers(-2**63, 2**63 - 1, 1000, dtype=np.int64),
                        np.array([0, 2**63 - 1, -1, -2**63, 7, 1 << 62], np.int64)])
    x, y, t = Z3SFC(period).invert(z)
    ox, oy, ot = oracle.z3_invert_batch(z, period)
    assert np.array_equal(f64_bits(as_np(x)), f64_bits(ox))
    assert np.array_equal(f64_bits(as_np(y)), f64_bits(oy))
    assert np.array_equal(as_np(t), ot)


@pytest.mark.parametrize("lenient", [False, True])
def test_z2_index_invert_parity(gpu, oracle, lenient):
    from geomesa_amd.curve import Z2SFC
    x, y, _ = random_points(200_001)
    ex, ey, _ = edge_points()
    x = np.concatenate([x, ex]); y = np.concatenate([y, ey])
    z, s = Z2SFC().index(x, y, lenient=lenient, status=True)
    oz, os_ = oracle.z2_index_batch(x, y, lenient)
    assert np.array_equal(as_np(s), os_) and np.array_equal(as_np(z), oz)
    rng = np.random.default_rng(3)
    zz = np.concatenate([oz, rng.integers(-2**63, 2**63 - 1, 10_000, dtype=np.int64)])
    ix, iy = Z2SFC().invert(zz)
    ox, oy = oracle.z2_invert_batch(zz)
    assert np.array_equal(f64_bits(as_np(ix)), f64_bits(ox)) and np.array_equal(f64_bits(as_np(iy)), f64_bits(oy))


def test_z2sfc_golden_values_gpu(gpu):  # geomesa-z3/src/test/.../zorder/sfcurve/Z2Test.scala:74-85
    from test_oracle_kats import Z2_GOLDEN
    from geomesa_amd.curve import Z2SFC
    xs = [float(p[0][0]) for p in Z2_GOLDEN]; ys = [float(p[0][1]) for p in Z2_GOLDEN]
    assert as_np(Z2SFC().index(xs, ys)).tolist() == [p[1] for p in Z2_GOLDEN]


@pytest.mark.parametrize("period", [0, 1, 2, 3])
def test_binned_time_parity(gpu, oracle, period):
    from geomesa_amd.curve import BinnedTime
    rng = np.random.default_rng(5)
    t = np.concatenate([rng.integers(-10**9, 2**45, 100_000), edge_points()[2]]).astype(np.int64)
    b, o, s = BinnedTime.time_to_binned_time(period, t, status=True)
    b, o, s = as_np(b), as_np(o), as_np(s)
    for i in range(0, len(t), 53):
        st, ob, oo = oracle.binned_time(period, int(t[i]))
        assert (s[i], b[i], o[i]) == (st, ob, oo)


def xz_envelopes(n, dims, seed=9):
    rng = np.random.default_rng(seed)
    cx = rng.uniform(-180, 180, n); cy = rng.uniform(-90, 90, n)
    w = 10 ** rng.uniform(-6, 1, n); h = 10 ** rng.uniform(-6, 1, n)
    env = [np.clip(cx - w, -180, 180), np.clip(cy - h, -90, 90), np.clip(cx + w, -180, 180), np.clip(cy + h, -90, 90)]
    # maxDim exactly / nearly a power of two
    k = rng.integers(1, 12, n // 8)
    base = np.full(n // 8, -100.0)
    env[0][: n // 8] = base; env[2][: n // 8] = base + 360.0 * np.ldexp(1.0, -k) * \
        rng.choice([1.0, 1 + 2**-40, 1 - 2**-40, 1 + 2**-52], n // 8)
    env[1][: n // 8] = 0.0; env[3][: n // 8] = 0.0
    if dims == 3:
        z0 = rng.uniform(0, 604800, n); dz = 10 ** rng.uniform(-3, 5.5, n)
        return [env[0], env[1], z0, env[2], env[3], np.clip(z0 + dz, 0, 604800)]
    return env


@pytest.mark.parametrize("lenient", [False, True])
def test_xz2_index_parity(gpu, oracle, lenient):
    from conftest import load_geoms
    from geomesa_amd.curve import XZ2SFC
    env = xz_envelopes(40_000, 2)
    g = np.array(load_geoms())
    env = [np.concatenate([e, g[:, k], [0.0, 190.0, 5.0]]) for k, e in enumerate(env)]
    env[2][-1] = 1.0  # unordered
    out, s = XZ2SFC(12).index(*env, lenient=lenient, status=True)
    oo, os_ = oracle.xz2_index_batch(np.stack(env, 1), lenient)
    assert np.array_equal(as_np(s), os_) and np.array_equal(as_np(out), oo)
    # misaligned device views (one row in) take the scalar kernel
    import torch
    dev = [torch.from_numpy(e).cuda()[1:] for e in env]
    out1, s1 = XZ2SFC(12).index(*dev, lenient=lenient, status=True)
    assert np.array_equal(as_np(s1), os_[1:]) and np.array_equal(as_np(out1), oo[1:])


@pytest.mark.parametrize("lenient", [False, True])
def test_xz3_index_parity(gpu, oracle, lenient):
    from geomesa_amd.curve import XZ3SFC
    env = xz_envelopes(40_000, 3)
    out, s = XZ3SFC(12, "week").index(*env, lenient=lenient, status=True)
    oo, os_ = oracle.xz3_index_batch(np.stack(env, 1), lenient)
    assert np.array_equal(as_np(s), os_) and np.array_equal(as_np(out), oo)
    import torch
    dev = [torch.from_numpy(e).cuda()[1:] for e in env]
    out1, s1 = XZ3SFC(12, "week").index(*dev, lenient=lenient, status=True)
    assert np.array_equal(as_np(s1), os_[1:]) and np.array_equal(as_np(out1), oo[1:])


def _ulp_walk(v, k):
    """v moved k ulps (k < 0: down)."""
    out = np.asarray(v, np.float64).copy()
    for _ in range(abs(k)):
        out = np.nextafter(out, np.inf if k > 0 else -np.inf)
    return out


def _division_edges(lo, span, rng, n_mult=4096):
    """values v in [lo, lo + span] whose normalized (v - lo) / span sits on or next to a dyadic boundary
    j / 2^20 (the cells floor((v - lo) / span * 2^L) turns on), plus the span's ends"""
    j = rng.integers(0, 2**20 + 1, n_mult)
    base = lo + np.ldexp(j.astype(np.float64), -20) * span
    vals = [base] + [_ulp_walk(base, k) for k in (-3, -2, -1, 1, 2, 3)] + [np.array([lo, lo + span])]
    return np.clip(np.concatenate(vals), lo, lo + span)


@pytest.mark.parametrize("g", [12, 20])
def test_xz_division_edges(gpu, oracle, g):
    """The XZ keys divide by the lon / lat / time spans with a corrected reciprocal (gm_keys.hpp div_span,
    div_time): degenerate and tiny envelopes whose normalized corners sit on, or 1-3 ulps beside, the
    dyadic cell boundaries, z = 0, subnormal, around 2^-900 (the IEEE fallback's edge) and integer
    offsets, for every period's span -- bit-equal keys with the oracle's IEEE division"""
    from geomesa_amd.curve import XZ2SFC, XZ3SFC
    rng = np.random.default_rng(17)
    xs = _division_edges(-180.0, 360.0, rng); ys = _division_edges(-90.0, 180.0, rng)
    n = max(len(xs), len(ys))
    xs = np.resize(xs, n); ys = np.resize(rng.permutation(ys), n)
    w = np.where(rng.random(n) < 0.5, 0.0, np.ldexp(1.0, -rng.integers(8, 40, n)))
    env2 = [xs, ys, np.minimum(xs + w, 180.0), np.minimum(ys + w, 90.0)]
    out, st = XZ2SFC(g).index(*env2, status=True)
    oo, ost = oracle.xz2_index_batch(np.stack(env2, 1), g=g)
    assert np.array_equal(as_np(st), ost) and np.array_equal(as_np(out), oo)
    if g > 20:
        return
    for name, period in (("day", oracle.DAY), ("week", oracle.WEEK), ("month", oracle.MONTH), ("year", oracle.YEAR)):
        span = float(XZ3SFC(g, name).zBounds[1])
        special = np.array([0.0, 5e-324, 1e-310, 2.2250738585072014e-308, np.ldexp(1.0, -1000),
                            np.ldexp(1.0, -900), np.nextafter(np.ldexp(1.0, -900), 0.0),
                            np.nextafter(np.ldexp(1.0, -900), 1.0), 1.0, span - 1.0, span])
        ints = rng.integers(0, int(span) + 1, 4096).astype(np.float64)
        zs = np.resize(np.concatenate([_division_edges(0.0, span, rng), special, ints]), n)
        zs = rng.permutation(zs)
        dz = np.where(rng.random(n) < 0.5, 0.0, np.ldexp(span, -rng.integers(8, 40, n)))
        env3 = [xs, ys, zs, env2[2], env2[3], np.minimum(zs + dz, span)]
        out, st = XZ3SFC(g, name).index(*env3, status=True)
        oo, ost = oracle.xz3_index_batch(np.stack(env3, 1), g=g, period=period)
        assert np.array_equal(as_np(st), ost), name
        assert np.array_equal(as_np(out), oo), name


def test_z3_roundtrip_property_large(gpu):
    """Size-independent property at 2^26 points: invert(z) returns the centre of z's lon/lat cell, so
    re-encoding it reproduces z's lon/lat bits (encode -> invert -> encode idempotence; the time
    dimension is truncated to whole seconds by Z3SFC.invert's .toLong and is excluded)."""
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.curve import Z3SFC
    n = 1 << 26
    ctx = _lib.context()
    x = torch.empty(n, dtype=torch.float64, device="cuda"); y = torch.empty_like(x)
    t = torch.empty(n, dtype=torch.int64, device="cuda")
    _lib.check(ctx.lib.gm_gen_points(ctx.handle, SEED, n, 0, -180.0, 180.0, -90.0, 90.0, T2020, T2021,
                                     _lib.ptr(x), _lib.ptr(y), _lib.ptr(t)), "gen")
    sfc = Z3SFC("week")
    b, z = sfc.index_keys(x, y, t)
    ix, iy, it = sfc.invert(z)
    z2 = sfc.index(ix, iy, it)
    mask_xy = ~0x4924924924924924
    assert torch.equal(z & mask_xy, z2 & mask_xy)
    assert int((b < 2608).sum()) == 0 and int((b > 2661).sum()) == 0
