"""GPU parity for the sorted key table: key bytes, table-order sort, and seek-and-filter range scans.

The expected table order is the store's byte order of [shard][bin BE16][z BE64]
(Z3IndexKeySpace.scala:81-92, ByteArrays.scala:51,90-99), computed here with a stable numpy lexsort
on the unsigned views; range scans are checked against the full-column Z3Filter scan (which the
oracle pins) and the Z3IdxStrategyTest KATs."""
import numpy as np
import pytest

from test_host_planning import IDX_STRATEGY_KATS, idx_strategy_features, ms
from geomesa_amd import filters as F
from geomesa_amd.keyspace import Z3IndexKeySpace, during

pytestmark = pytest.mark.gpu

T2020, T2021 = 1577836800000, 1609459200000


def as_np(t):
    return t.detach().cpu().numpy()


def expected_order(bins, z, shard=None):
    keys = [np.asarray(z).view(np.uint64), np.asarray(bins).view(np.uint16)]
    if shard is not None:
        keys.append(np.asarray(shard, np.uint8))
    return np.lexsort(keys)   # stable; last key is primary


@pytest.mark.parametrize("n,kind", [(1, "rand"), (2, "rand"), (2047, "rand"), (2049, "rand"), (300_001, "rand"),
                                    (100_000, "equal"), (100_000, "few"), (1_000_003, "keys"), (399_900, "dups"),
                                    (600_000, "narrow"), (200_000, "runs")])
@pytest.mark.parametrize("sharded", [False, True])
@pytest.mark.parametrize("mode", [0, 1])
def test_sort_keys_parity(gpu, n, kind, sharded, mode):
    """mode 0: prefix passes + local ranks (digit passes when a run of equal prefixes exceeds 256
    rows: unsharded "dups"); mode 1: digit passes over every varying byte (GM_PARAM_SORT_MODE)."""
    import torch
    from geomesa_amd import _lib
    rng = np.random.default_rng(n + sharded)
    if kind == "rand":     # every bit pattern: negative bins / z sort as unsigned bytes
        bins = rng.integers(-2**15, 2**15, n).astype(np.int16)
        z = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    elif kind == "equal":  # every digit pass skipped
        bins = np.full(n, 2610, np.int16); z = np.full(n, 123456789, np.int64)
    elif kind == "few":    # heavy duplicates: stability decides the permutation
        bins = rng.integers(2608, 2611, n).astype(np.int16); z = rng.integers(0, 5, n).astype(np.int64)
    elif kind == "dups":   # real keys, each repeated 300 times: runs longer than 256 rows
        x = rng.uniform(-180, 180, n // 300); y = rng.uniform(-90, 90, n // 300); t = rng.integers(T2020, T2021, n // 300)
        b, zz = Z3IndexKeySpace().sfc.index_keys(x, y, t)
        idx = rng.permutation(np.repeat(np.arange(n // 300), 300))
        bins, z = as_np(b)[idx], as_np(zz)[idx]
    elif kind == "narrow":  # one bin, 40 varying z bits: the prefix window straddles no column
        bins = np.full(n, -7, np.int16); z = rng.integers(0, 2**40, n, dtype=np.int64)
    elif kind == "runs":   # runs of 1-48 equal prefixes with distinct low bits (ranked locally, ties included)
        pre = np.repeat(rng.choice(2**24, 12000, replace=False), rng.integers(1, 49, 12000))[:n].astype(np.int64)
        rng.shuffle(pre)
        bins = (pre >> 12).astype(np.int16)
        z = ((pre & 0xfff) << 52) | rng.integers(0, 8, n, dtype=np.int64)   # bits 52-63 (negative z included)
    else:                  # real keys
        x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n); t = rng.integers(T2020, T2021, n)
        b, zz = Z3IndexKeySpace().sfc.index_keys(x, y, t)
        bins, z = as_np(b), as_np(zz)
    shard = rng.integers(0, 4, n).astype(np.uint8) if sharded else None
    ctx = _lib.context()
    ctx.set_param(_lib.GM_PARAM_SORT_MODE, mode)
    db, dz = torch.from_numpy(bins).cuda(), torch.from_numpy(z).cuda()
    ds = torch.from_numpy(shard).cuda() if sharded else None
    ob, oz, op = torch.empty_like(db), torch.empty_like(dz), torch.empty(n, dtype=torch.int64, device="cuda")
    os_ = torch.empty_like(ds) if sharded else None
    _lib.check(ctx.lib.gm_sort_keys(ctx.handle, _lib.ptr(ds), _lib.ptr(db), _lib.ptr(dz), n, _lib.ptr(os_),
                                    _lib.ptr(ob), _lib.ptr(oz), _lib.ptr(op)), "sort")
    order = expected_order(bins, z, shard)
    assert np.array_equal(as_np(op), order)
    assert np.array_equal(as_np(ob), bins[order]) and np.array_equal(as_np(oz), z[order])
    if sharded:
        assert np.array_equal(as_np(os_), shard[order])
    last = ctx.get_param(_lib.GM_PARAM_SORT_LAST)
    ctx.set_param(_lib.GM_PARAM_SORT_MODE, 0)
    if mode == 1:
        assert last < 256
    elif kind in ("rand", "keys", "narrow", "runs") and n > 100_000:
        assert last > 256, last               # prefix passes + local ranks
    elif kind == "dups" and not sharded:
        assert last < 256 and last > 3, last  # runs > 256 rows: digit passes
    elif kind == "dups":
        assert last > 256, last               # 4 shards split each 300-row run into ~75: ranked locally


def _check_table_order_on_device(bins, z, ob, oz, op, sh=None, osh=None):
    """Device-side checks of a large sort: output = input[perm], perm a permutation, keys
    nondecreasing in (shard, bin unsigned, z unsigned) order, and stable (equal keys keep input
    order)."""
    import torch
    n = z.numel()
    assert torch.equal(ob, bins[op]) and torch.equal(oz, z[op])
    if sh is not None:
        assert torch.equal(osh, sh[op])
    seen = torch.zeros(n, dtype=torch.bool, device=z.device)
    seen[op] = True
    assert bool(seen.all())
    hi = (ob.to(torch.int64) & 0xFFFF) | ((osh.to(torch.int64) << 16) if osh is not None else 0)
    lo = oz ^ (-(1 << 63))   # unsigned order as signed
    dh, dl = hi[1:] - hi[:-1], lo[1:] - lo[:-1]
    le = (dh > 0) | ((dh == 0) & (lo[1:] >= lo[:-1]))
    assert bool(le.all())
    tie = (dh == 0) & (dl == 0)
    assert bool((op[1:][tie] > op[:-1][tie]).all())


@pytest.mark.parametrize("kind", ["week_keys", "dups", "sharded"])
def test_sort_keys_prefix_path_at_bench_size(gpu, kind):
    """The bench's sort path (2^27 < n: three 9-bit prefix digits + local ranks) on 140M rows: Z3 keys
    of uniform points over 2020 (53 weekly bins, runs of equal prefixes of a few rows), the same
    keys with every key repeated 4 times (ties: stability), and the keys with GeoMesa's default 4
    shards (geomesa.z.splits, Conversions.scala:312): the shard sits right above bin's varying bits in
    the sort key, so the prefix digits still cover ~log2(n) varying bits and the local ranks run
    (a digit spanning bin's constant top bits sent this case to 3x the time); checked on the device."""
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.curve import Z3SFC
    n = 140_000_000
    g = torch.Generator(device="cuda").manual_seed(3)
    m = n // 4 if kind == "dups" else n
    x = torch.rand(m, device="cuda", generator=g, dtype=torch.float64) * 360 - 180
    y = torch.rand(m, device="cuda", generator=g, dtype=torch.float64) * 180 - 90
    t = (torch.rand(m, device="cuda", generator=g, dtype=torch.float64) * 31622400000).to(torch.int64) + T2020
    b, z = Z3SFC("week").index_keys(x, y, t)
    del x, y, t
    if kind == "dups":
        idx = torch.randperm(n, device="cuda", generator=g) % m
        b, z = b[idx].contiguous(), z[idx].contiguous()
        del idx
    sh = osh = None
    if kind == "sharded":
        sh = torch.randint(0, 4, (n,), device="cuda", generator=g, dtype=torch.uint8)
        osh = torch.empty_like(sh)
    ob, oz = torch.empty_like(b), torch.empty_like(z)
    op = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = _lib.context()
    _lib.check(ctx.lib.gm_sort_keys(ctx.handle, _lib.ptr(sh), _lib.ptr(b), _lib.ptr(z), n, _lib.ptr(osh), _lib.ptr(ob),
                                    _lib.ptr(oz), _lib.ptr(op)), "sort")
    assert ctx.get_param(_lib.GM_PARAM_SORT_LAST) == 256 + 3   # three prefix passes + local ranks
    _check_table_order_on_device(b, z, ob, oz, op, sh, osh)


def test_sort_keys_prefix_keeps_first_digit_top_bits(gpu):
    """n in (2^25, 2^28]: three 9-bit prefix digits.  The only varying bits of the first digit are its
    top four (z bits 59-62); the other two digits see 16 varying bits (z bits 16-31), so a prefix that
    dropped the first digit's top bits would merge 16 runs into one of ~512 rows, past RUN_MAX, and send
    the sort down the every-byte fallback.  The prefix keeps them: the local-rank path runs."""
    import torch
    from geomesa_amd import _lib
    n = (1 << 25) + 4096
    g = torch.Generator(device="cuda").manual_seed(5)
    top = torch.randint(0, 16, (n,), device="cuda", generator=g, dtype=torch.int64) << 59
    mid = torch.randint(0, 1 << 16, (n,), device="cuda", generator=g, dtype=torch.int64) << 16
    low = torch.randint(0, 2, (n,), device="cuda", generator=g, dtype=torch.int64)
    z = top | mid | low
    b = torch.full((n,), 2610, dtype=torch.int16, device="cuda")
    del top, mid, low
    ob, oz = torch.empty_like(b), torch.empty_like(z)
    op = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = _lib.context()
    _lib.check(ctx.lib.gm_sort_keys(ctx.handle, None, _lib.ptr(b), _lib.ptr(z), n, None, _lib.ptr(ob), _lib.ptr(oz),
                                    _lib.ptr(op)), "sort")
    assert ctx.get_param(_lib.GM_PARAM_SORT_LAST) == 256 + 3
    _check_table_order_on_device(b, z, ob, oz, op)


@pytest.mark.parametrize("where", ["bin", "shard", "z"])
@pytest.mark.parametrize("mode", [0, 1])
def test_sort_keys_sample_misses_a_varying_bit(gpu, where, mode):
    """The digits are planned from the OR / AND of a strided sample (every (n // 65536)-th row and
    the last) and counted in the read that takes the exact OR / AND; here the highest varying bit
    changes in one row the sample skips, so the exact plan differs and the digits are counted again."""
    import torch
    from geomesa_amd import _lib
    n, odd = 1_000_003, 500_001
    assert odd % (n // 65536) != 0
    rng = np.random.default_rng(11)
    bins = np.full(n, 2610, np.int16)
    z = rng.integers(0, 2**40, n, dtype=np.int64)
    shard = np.full(n, 2, np.uint8)
    if where == "bin":
        bins[odd] = 2700
    elif where == "shard":
        shard[odd] = 3
    else:
        z[odd] |= 1 << 62
    ctx = _lib.context()
    ctx.set_param(_lib.GM_PARAM_SORT_MODE, mode)
    db, dz, ds = torch.from_numpy(bins).cuda(), torch.from_numpy(z).cuda(), torch.from_numpy(shard).cuda()
    ob, oz, os_ = torch.empty_like(db), torch.empty_like(dz), torch.empty_like(ds)
    op = torch.empty(n, dtype=torch.int64, device="cuda")
    _lib.check(ctx.lib.gm_sort_keys(ctx.handle, _lib.ptr(ds), _lib.ptr(db), _lib.ptr(dz), n, _lib.ptr(os_),
                                    _lib.ptr(ob), _lib.ptr(oz), _lib.ptr(op)), "sort")
    ctx.set_param(_lib.GM_PARAM_SORT_MODE, 0)
    order = expected_order(bins, z, shard)
    assert np.array_equal(as_np(op), order)
    assert np.array_equal(as_np(ob), bins[order]) and np.array_equal(as_np(oz), z[order])
    assert np.array_equal(as_np(os_), shard[order])
    assert as_np(op)[-1] == odd   # the one key with the highest varying bit set sorts last


@pytest.mark.parametrize("in_off,out_off", [(1, 0), (0, 1), (1, 3)])
def test_sort_keys_unaligned_columns(gpu, in_off, out_off):
    """Caller columns off the 16-B grid (slices): the pair-load paths must not be taken for them."""
    import torch
    from geomesa_amd import _lib
    n = 150_001
    rng = np.random.default_rng(11)
    bins = rng.integers(-2**15, 2**15, n).astype(np.int16)
    z = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    shard = rng.integers(0, 3, n).astype(np.uint8)
    pad = lambda a, o: torch.from_numpy(np.concatenate([np.zeros(o, a.dtype), a])).cuda()[o:]
    db, dz, ds = pad(bins, in_off), pad(z, in_off), pad(shard, in_off)
    ob = torch.empty(n + out_off, dtype=torch.int16, device="cuda")[out_off:]
    oz = torch.empty(n + out_off, dtype=torch.int64, device="cuda")[out_off:]
    os_ = torch.empty(n + out_off, dtype=torch.uint8, device="cuda")[out_off:]
    op = torch.empty(n, dtype=torch.int64, device="cuda")
    ctx = _lib.context()
    _lib.check(ctx.lib.gm_sort_keys(ctx.handle, _lib.ptr(ds), _lib.ptr(db), _lib.ptr(dz), n, _lib.ptr(os_),
                                    _lib.ptr(ob), _lib.ptr(oz), _lib.ptr(op)), "sort")
    order = expected_order(bins, z, shard)
    assert np.array_equal(as_np(op), order)
    assert np.array_equal(as_np(ob), bins[order]) and np.array_equal(as_np(oz), z[order])
    assert np.array_equal(as_np(os_), shard[order])


@pytest.mark.parametrize("sharded", [False, True])
def test_key_bytes(gpu, sharded):
    from geomesa_amd.table import Z3Table
    rng = np.random.default_rng(5)
    n = 70_001
    bins = rng.integers(-2**15, 2**15, n).astype(np.int16)
    z = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64, endpoint=True)
    shard = rng.integers(0, 4, n).astype(np.uint8) if sharded else None
    tb = Z3Table(bins, z, shard)
    kb = as_np(tb.key_bytes())
    order = expected_order(bins, z, shard)
    exp = Z3IndexKeySpace.key_bytes(bins[order], z[order], None if shard is None else shard[order])
    assert np.array_equal(kb, exp)
    # table order is the byte order of the keys (what Accumulo / HBase keep sorted)
    rows = [bytes(r) for r in kb[:: 97]]
    assert rows == sorted(rows)


@pytest.mark.parametrize("bbox,interval,expected", IDX_STRATEGY_KATS)
def test_table_query_idx_strategy_kats(gpu, bbox, interval, expected):  # Z3IdxStrategyTest.scala:96-181
    from geomesa_amd.table import Z3Table
    feats = idx_strategy_features()
    ids = np.array([f[0] for f in feats])
    tb = Z3Table.from_points([f[1] for f in feats], [f[2] for f in feats], [f[3] for f in feats])
    got, n, scanned = tb.query([bbox], [interval])
    assert set(ids[as_np(got)].tolist()) == expected and n == len(expected) and scanned >= n


def random_points(n, seed):
    rng = np.random.default_rng(seed)
    return rng.uniform(-180, 180, n), rng.uniform(-90, 90, n), rng.integers(T2020, T2021, n)


QUERIES = [
    ([(-10, 35, 30, 60)], [during(ms("2020-06-01T00:00:00.000Z"), ms("2020-06-08T12:00:00.000Z"))]),
    ([(-10, 35, 30, 60), (100, -40, 120, -10)], [during(ms("2020-03-01T00:00:00.000Z"),
                                                        ms("2020-05-08T12:00:00.000Z"))]),
    ([(0.0, 0.0, 0.5, 0.5)], [during(ms("2020-01-01T00:00:00.000Z"), ms("2020-01-09T00:00:00.500Z"))]),
    ([(-180, -90, 180, 90)], [during(ms("2020-12-30T00:00:00.000Z"), ms("2021-01-01T00:00:00.000Z"))]),
    ([(-50, -50, 50, 50)], None),   # no time predicate: one unbounded range
]


@pytest.mark.parametrize("q", range(len(QUERIES)))
@pytest.mark.parametrize("sharded", [False, True])
def test_table_query_equals_full_scan(gpu, oracle, q, sharded):
    """Seek-and-filter over the sorted table returns exactly the rows of a full-column scan with
    the same Z3Filter and epoch restriction (the claim of SURVEY 8(e)), which the oracle pins."""
    from geomesa_amd.table import Z3Table
    x, y, t = random_points(1_000_003, seed=40 + q)
    shard = np.arange(len(x)) % 4 if sharded else None
    ks = Z3IndexKeySpace()
    b, z = ks.sfc.index_keys(x, y, t)
    tb = Z3Table(b, z, shard)
    bb, iv = QUERIES[q]
    got, n, scanned = tb.query(bb, iv)
    v = ks.get_index_values(bb, iv)
    f = F.Z3Filter.from_values(v)
    om = oracle.z3filter_scan(F.serialize_to_bytes(f), ks.bin_ranges(v), as_np(b), as_np(z))
    assert n == int(om.sum()) and np.array_equal(np.sort(as_np(got)), np.nonzero(om)[0])
    assert scanned >= n and (q == 4 or scanned < len(x) // 4)   # the ranges prune
    # table-order ids are ascending
    tid, n2, _ = tb.scan(ks.get_ranges(v), f, map_rows=False)
    assert n2 == n and np.all(np.diff(as_np(tid)) > 0)


def test_table_scan_open_ranges_and_capacity(gpu):
    """Lower/upper-bounded and unbounded scan ranges (after / before predicates), overlapping ranges
    merged as a BatchScanner does, and the GM_E_CAPACITY path."""
    from geomesa_amd.table import Z3Table
    x, y, t = random_points(200_001, seed=3)
    ks = Z3IndexKeySpace()
    b, z = ks.sfc.index_keys(x, y, t)
    tb = Z3Table(b, z)
    bn, zn = as_np(b).astype(np.int64), as_np(z)
    keys = as_np(b).view(np.uint16).astype(np.int64)   # bins compare as unsigned bytes
    for kind, lo, hi, sel in [
            ("lower", (2630, 0), None, keys >= 2630),
            ("upper", None, (2620, 2**63 - 1), keys <= 2620),
            ("unbounded", (0, 0), None, np.ones(len(keys), bool))]:
        got, n, scanned = tb.scan([(kind, lo, hi)], None)
        assert n == int(sel.sum()) == scanned and np.array_equal(np.sort(as_np(got)), np.nonzero(sel)[0])
    # overlapping bounded ranges scan each row once
    zs = np.sort(zn[bn == 2640])
    r1 = ("bounded", (2640, int(zs[10])), (2640, int(zs[500])))
    r2 = ("bounded", (2640, int(zs[300])), (2640, int(zs[900])))
    got, n, scanned = tb.scan([r1, r2, r1], None)
    exp = np.nonzero((bn == 2640) & (zn >= zs[10]) & (zn <= zs[900]))[0]
    assert n == len(exp) == scanned and np.array_equal(np.sort(as_np(got)), exp)
    got, n, _ = tb.scan([r1, r2], None, ids_cap=7)
    assert n == len(exp) and len(got) == 7
    # empty table / no ranges
    assert tb.scan([], None)[1] == 0


# ---------------------------------------------------------------- key-range partition (multi-GPU ingest)

def _partition_keys(rng, n, kind):
    sh = rng.integers(0, 4, n).astype(np.uint8)
    if kind == "rand":
        b = rng.choice(np.array([0, 1, 2600, 32767, -32768, -2], np.int16), n)
        z = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64, endpoint=True)
    elif kind == "week":
        x, y = rng.uniform(-180, 180, n), rng.uniform(-90, 90, n)
        t = rng.integers(T2020, T2021, n)
        from geomesa_amd.curve import Z3SFC
        bb, zz = Z3SFC("week").index_keys(x, y, t)
        b, z = as_np(bb), as_np(zz)
    else:   # "dups": few distinct keys, many equal to a splitter
        b = rng.integers(0, 3, n).astype(np.int16)
        z = rng.integers(0, 5, n).astype(np.int64)
    return sh, b, z


@pytest.mark.parametrize("n", [0, 1, 2048, 2049, 100_003, 1_000_000])
@pytest.mark.parametrize("kind", ["rand", "week", "dups"])
@pytest.mark.parametrize("nd", [1, 3, 8, 17])
@pytest.mark.parametrize("sharded", [False, True])
def test_key_partition_equals_oracle(gpu, oracle, n, kind, nd, sharded):
    """gm_key_partition against its definition (oracle.key_partition): the output columns are the input
    rows in destination-then-input order, the sources (ids column, id_base + row, 4-B rows) follow, and
    the counts match.  Splitters are drawn from the keys (so keys equal a splitter) and repeated."""
    if kind == "rand" and n > 100_003 and nd > 3:
        pytest.skip("covered by the smaller random cases")
    import torch
    from geomesa_amd import shard as S
    rng = np.random.default_rng(n * 31 + nd * 7 + sharded)
    sh, b, z = _partition_keys(rng, n, kind)
    hi, lo = oracle.table_key_u64(sh if sharded else None, b, z)
    if n:
        pick = np.sort(rng.integers(0, n, nd - 1))
        keys = sorted(zip(hi[pick].tolist(), lo[pick].tolist()))
        if nd > 2:
            keys[1] = keys[0]
    else:
        keys = sorted((int(rng.integers(0, 1 << 24)), int(rng.integers(0, 1 << 62))) for _ in range(nd - 1))
    sp_hi = np.array([k[0] for k in keys], np.uint64)
    sp_lo = np.array([k[1] for k in keys], np.uint64)
    order, counts = oracle.key_partition(sh if sharded else None, b, z, sp_hi, sp_lo)
    dev = gpu.device
    tsh = torch.from_numpy(sh).cuda(dev) if sharded else None
    tb, tz = torch.from_numpy(b).cuda(dev), torch.from_numpy(z).cuda(dev)
    ids = rng.integers(-(1 << 62), 1 << 62, n).astype(np.int64)
    for mode in ("ids", "base", "rows"):
        cols, got = S.partition_rows(gpu, tsh, tb, tz, sp_hi, sp_lo,
                                     ids=torch.from_numpy(ids).cuda(dev) if mode == "ids" else None,
                                     id_base=12345, rows=mode == "rows")
        assert got == counts.tolist()
        src = as_np(cols[-1])
        if sharded:
            assert np.array_equal(as_np(cols[0]), sh[order])
        assert np.array_equal(as_np(cols[-3]), b[order]) and np.array_equal(as_np(cols[-2]), z[order])
        exp = {"ids": ids[order], "base": order + 12345, "rows": order.astype(np.int32)}[mode]
        assert np.array_equal(src, exp), mode


def test_key_partition_rejects_bad_splitters(gpu):
    import ctypes
    import torch
    from geomesa_amd import _lib
    z = torch.arange(10, dtype=torch.int64, device="cuda")
    b = torch.zeros(10, dtype=torch.int16, device="cuda")
    out_b, out_z = torch.empty_like(b), torch.empty_like(z)
    cnt = np.zeros(3, np.int64)
    P = _lib.ptr
    for hi, lo in (([1, 0], [0, 0]), ([0, 0], [5, 4]), ([1 << 24, 1 << 24], [0, 0])):
        h, lo_ = np.array(hi, np.uint64), np.array(lo, np.uint64)
        rc = gpu.lib.gm_key_partition(gpu.handle, None, P(b), P(z), 10, h.ctypes.data, lo_.ctypes.data, 2, None, 0,
                                      None, P(out_b), P(out_z), None, None, cnt.ctypes.data)
        assert rc == _lib.GM_E_INVALID
    big = np.zeros(256, np.uint64)
    assert gpu.lib.gm_key_partition(gpu.handle, None, P(b), P(z), 10, big.ctypes.data, big.ctypes.data, 256, None, 0,
                                    None, P(out_b), P(out_z), None, None, np.zeros(257, np.int64).ctypes.data) \
        == _lib.GM_E_INVALID
    del ctypes


@pytest.mark.parametrize("n,k", [(1, 1), (1000, 64), (1_000_003, 1024), (70_000, 65536)])
@pytest.mark.parametrize("sharded", [False, True])
def test_key_sample(gpu, oracle, n, k, sharded):
    import torch
    from geomesa_amd import shard as S
    rng = np.random.default_rng(n + k)
    sh, b, z = _partition_keys(rng, n, "rand")
    hi, lo = S.sample_keys(gpu, torch.from_numpy(sh).cuda() if sharded else None, torch.from_numpy(b).cuda(),
                           torch.from_numpy(z).cuda(), k)
    rows = (2 * np.arange(k, dtype=np.int64) + 1) * n // (2 * k)
    eh, el = oracle.table_key_u64(sh if sharded else None, b, z)
    assert np.array_equal(hi, eh[rows]) and np.array_equal(lo, el[rows])
