"""Multi-process (gloo, world_size 2, CPU) tests of the sharding path bench.py and users run over RCCL.

The product kernels need the GPU, so the per-rank compute here is the C oracle (test
infrastructure): what is checked is the distributed bookkeeping -- shard bounds, the polygon-set
broadcast, id_base offsets of per-rank join output, and the max/sum reductions -- which is the same
code the RCCL path runs.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from geomesa_amd.join import synthetic_counties, synthetic_points
        import torch
        from geomesa_amd.shard import all_reduce_scalar, broadcast_polyset, gather_rows, shard_bounds
        ps = synthetic_counties(20, 10) if rank == 0 else None
        ps = broadcast_polyset(dist, ps)
        px, py = synthetic_points(n_total, seed=21)
        lo, hi = shard_bounds(n_total, rank, world)
        pt, pl = O.OraclePolySet(*ps.to_arrays()).join(px[lo:hi], py[lo:hi], nthreads=2)
        if rank == 1:   # unequal per-rank counts exercise the padded gather
            pt, pl = pt[: len(pt) // 2], pl[: len(pl) // 2]
        g = gather_rows(dist, [torch.from_numpy(pt + lo), torch.from_numpy(pl.astype(np.int32))])
        tot = all_reduce_scalar(dist, len(pt), "sum")
        mx = all_reduce_scalar(dist, float(rank + 1), "max")
        if rank == 0:
            pairs = np.stack([g[0].numpy(), g[1].numpy().astype(np.int64)], 1)
            q.put((pairs, tot, mx, ps.vx.sum(), ps.n_polys))
        else:
            assert g is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_join_equals_global(world, oracle):
    from geomesa_amd.join import synthetic_counties, synthetic_points
    n_total = 60_001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got, tot, mx, vxsum, npoly = res
    ps = synthetic_counties(20, 10)
    assert npoly == ps.n_polys and vxsum == ps.vx.sum()      # broadcast delivered the same set
    px, py = synthetic_points(n_total, seed=21)
    from geomesa_amd.shard import shard_bounds
    exp = []
    for r in range(world):   # each rank's shard joined alone (rank 1 keeps half its pairs)
        lo, hi = shard_bounds(n_total, r, world)
        opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px[lo:hi], py[lo:hi], nthreads=4)
        if r == 1:
            opt, opl = opt[: len(opt) // 2], opl[: len(opl) // 2]
        exp.append(np.stack([opt + lo, opl.astype(np.int64)], 1))
    exp = np.concatenate(exp)
    assert np.array_equal(got, exp)             # rank order, each rank's order kept
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    got = got[np.lexsort((got[:, 1], got[:, 0]))]
    assert np.array_equal(got, exp)
    assert tot == len(exp) and mx == float(world)


def test_shard_bounds():
    from geomesa_amd.shard import shard_bounds
    for n in (0, 1, 7, 1000, 10**9 + 3):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def _hist_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from geomesa_amd.shard import merge_histograms, shard_bounds
        import torch
        x, y, t = _hist_points()
        lo, hi = shard_bounds(len(x), rank, world)
        b, _, st = O.z3_index_key_batch(x[lo:hi], y[lo:hi], t[lo:hi])
        blo, bhi = int(b[st == 0].min()), int(b[st == 0].max())   # each rank its own window
        pres, counts, _ = O.z3_histogram(x[lo:hi], y[lo:hi], t[lo:hi], 64, blo, bhi - blo + 1)
        c, p, mlo = merge_histograms(dist, torch.from_numpy(counts), torch.from_numpy(pres), blo)
        if rank == 0:
            q.put((c.numpy(), p.numpy(), mlo))
    finally:
        dist.destroy_process_group()


def _hist_points():
    rng = np.random.default_rng(5)
    n = 40_001
    x = rng.uniform(-180, 180, n); y = rng.uniform(-90, 90, n)
    t = np.sort(rng.integers(1577836800000, 1609459200000, n))   # sorted: ranks see different weeks
    x[7] = 200.0                                                  # one toKey failure
    return x, y, t


def test_sharded_histogram_merge_equals_global(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hist_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    c, p, mlo = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    x, y, t = _hist_points()
    pres, counts, tally = oracle.z3_histogram(x, y, t, 64, mlo, c.shape[0])
    assert tally.tolist() == [1, 0]
    assert np.array_equal(c, counts) and np.array_equal(p, pres)


def _hist_mismatch_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from geomesa_amd.shard import merge_histograms
        length = 64 if rank == 0 else 32          # Z3Histogram += of different lengths throws
        counts = torch.ones((3, length), dtype=torch.int64)
        pres = torch.ones(3, dtype=torch.uint8)
        try:
            merge_histograms(dist, counts, pres, 2600 + rank)
            q.put((rank, "no error"))
        except NotImplementedError as e:
            q.put((rank, str(e)))
        # the group is still usable: no rank is left inside a collective
        t = torch.tensor([rank + 1.0])
        dist.all_reduce(t)
        q.put((rank, float(t.item())))
    finally:
        dist.destroy_process_group()


def test_histogram_merge_length_mismatch_raises_on_every_rank():
    """the length check happens on every rank before any tensor collective."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hist_mismatch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(2 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    msgs = sorted(m for m in got if isinstance(m[1], str))
    sums = [m for m in got if not isinstance(m[1], str)]
    assert msgs == [(0, "Can only add z3 histograms with the same length"),
                    (1, "Can only add z3 histograms with the same length")]
    assert sorted(s[1] for s in sums) == [3.0, 3.0]


def test_merge_histograms_without_group():
    import torch
    from geomesa_amd.shard import merge_histograms
    c, p = torch.arange(6, dtype=torch.int64).reshape(2, 3), torch.tensor([1, 0], dtype=torch.uint8)
    rc, rp, lo = merge_histograms(None, c, p, 2600)
    assert rc is c and rp is p and lo == 2600
    assert merge_histograms(None, None, None, None) == (None, None, None)


# ---------------------------------------------------------------- key-range partitioned table (configs[2])

def _rand_keys(rng, n):
    """(shard, bin, z) rows with shards 0-3, bins on both sides of the unsigned-short sign flip and z
    spanning the whole unsigned range."""
    sh = rng.integers(0, 4, n).astype(np.uint8)
    b = rng.choice(np.array([0, 1, 2, 2600, 32767, -32768, -2], np.int16), n)
    z = rng.integers(-(1 << 63), (1 << 63) - 1, n, dtype=np.int64, endpoint=True)
    z[rng.random(n) < 0.3] = rng.integers(0, 50, int((rng.random(n) < 0.3).sum()) or 1)[0]
    return sh, b, z


def _order_key(sh, b, z):
    """Python tuple ordering = row-byte ordering (bin and z unsigned)."""
    return list(zip(sh.astype(int).tolist(), (b.astype(np.int64) & 0xffff).tolist(),
                    (z.astype(np.int64).view(np.uint64)).tolist()))


def test_clip_key_ranges_matches_brute_force():
    from geomesa_amd import _lib
    from geomesa_amd.shard import clip_key_ranges, table_key
    import torch
    rng = np.random.default_rng(3)
    sh, b, z = _rand_keys(rng, 3000)
    keys = _order_key(sh, b, z)
    skeys = sorted(keys)
    for trial in range(40):
        nr = 30
        arr = np.zeros(nr, _lib.KEY_RANGE_DTYPE)
        i = rng.integers(0, len(keys), (nr, 2))
        for k in range(nr):
            a, c = sorted([keys[i[k, 0]], keys[i[k, 1]]])
            if a[0] != c[0]:
                c = (a[0], 0xffff, (1 << 64) - 1)   # ranges stay inside one shard
            arr[k]["shard"] = a[0]
            arr[k]["bin_lo"], arr[k]["bin_hi"] = np.int64(a[1]).astype(np.int16), np.int64(c[1]).astype(np.int16)
            arr[k]["z_lo"], arr[k]["z_hi"] = np.uint64(a[2]).view(np.int64), np.uint64(c[2]).view(np.int64)
        lo_i, hi_i = sorted(rng.integers(0, len(skeys), 2))
        smin, smax = skeys[lo_i], skeys[hi_i]

        def tk(k):
            h, l_ = table_key(torch.tensor([k[0]], dtype=torch.uint8), torch.tensor([np.int64(k[1]).astype(np.int16)]),
                              torch.tensor([np.uint64(k[2]).view(np.int64)]))
            return int(h.item()), int(l_.item())
        out = clip_key_ranges(arr, tk(smin), tk(smax))

        def inside(rows, k):
            for r in rows:
                lo = (int(r["shard"]), int(r["bin_lo"]) & 0xffff, int(np.int64(r["z_lo"]).view(np.uint64)))
                hi = (int(r["shard"]), int(r["bin_hi"]) & 0xffff, int(np.int64(r["z_hi"]).view(np.uint64)))
                if lo <= k <= hi:
                    return True
            return False
        for k in keys:
            assert inside(out, k) == (inside(arr, k) and smin <= k <= smax), (trial, k)
        assert all(r["shard"] == r["shard"] for r in out)
    assert len(clip_key_ranges(arr, None, None)) == 0


def _sample_rows(n, k):
    """The rows gm_key_sample reads: floor((2i + 1) n / (2k))."""
    return (2 * np.arange(k, dtype=np.int64) + 1) * n // (2 * k)


def _xchg_worker(rank, world, port, sizes, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from geomesa_amd.shard import choose_splitters, exchange_partitioned
        rng = np.random.default_rng(100 + rank)
        sh, b, z = _rand_keys(rng, sizes[rank])          # unsorted rows, as every rank starts
        n, k = len(z), min(64, len(z))
        hi, lo = O.table_key_u64(sh, b, z)
        rows = _sample_rows(n, k)
        spl = choose_splitters(dist, hi[rows], lo[rows], n, samples=64)
        # the per-rank partition pass is the HIP kernel on the GPU; here its definition (the oracle)
        order, counts = O.key_partition(sh, b, z, *spl)
        gid = order.astype(np.int64) + rank * 10**6
        cols = [torch.from_numpy(np.ascontiguousarray(c[order])) for c in (sh, b, z)] + [torch.from_numpy(gid)]
        got, recv = exchange_partitioned(dist, cols, counts)
        s2, b2, z2, rg = (c.numpy() for c in got)
        q.put((rank, s2, b2, z2, rg, spl[0], spl[1], recv))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes", [(2, (5000, 3001)), (3, (4000, 0, 2500)),
                                         (8, (3000, 2000, 0, 4100, 1, 2500, 3333, 1800))])
def test_partition_exchange_by_key_range(world, sizes):
    """Splitters from every rank's UNSORTED sample, the stable partition, the per-column all-to-all: every
    row lands on the rank owning its key range, nothing is lost or duplicated, the ranges are ordered,
    the split is balanced (an empty rank included), and within each received slice the rows of one
    sender keep that sender's input order (what makes the receiver's one stable sort tie-break by id)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_xchg_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spl = list(zip(got[0][5].tolist(), got[0][6].tolist()))
    assert len(spl) == world - 1 and spl == sorted(spl)
    assert all(np.array_equal(g[5], got[0][5]) and np.array_equal(g[6], got[0][6]) for g in got)
    sent = []
    for r in range(world):
        rng = np.random.default_rng(100 + r)
        sh, b, z = _rand_keys(rng, sizes[r])
        sent += [(k, i + r * 10**6) for i, k in enumerate(_order_key(sh, b, z))]
    recv = []
    bounds = []
    for r, s2, b2, z2, rg, _, _, rc in got:
        assert sum(rc) == len(z2)
        ks = _order_key(s2, b2, z2)
        recv += list(zip(ks, rg.tolist()))
        bounds.append((min(ks), max(ks)) if ks else None)
        for kk in ks:   # key range of rank r: [splitter r-1, splitter r)
            key = (kk[0] << 16 | kk[1], kk[2])
            assert r == 0 or key >= spl[r - 1]
            assert r == world - 1 or key < spl[r]
        assert np.all(np.diff(rg // 10**6) >= 0)                       # senders in rank order
        for src in np.unique(rg // 10**6):
            assert np.all(np.diff(rg[rg // 10**6 == src]) > 0)          # each sender's rows in input order
    assert sorted(recv) == sorted(sent)
    nz = [bd for bd in bounds if bd]
    assert all(nz[i][1] <= nz[i + 1][0] for i in range(len(nz) - 1))
    n = sum(sizes)
    assert max(len(g[1]) for g in got) <= 1.35 * n / world


def test_key_partition_definition():
    """The oracle's partition: destination = number of splitters <= key, stable, counts per destination."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rng = np.random.default_rng(5)
    sh, b, z = _rand_keys(rng, 4000)
    hi, lo = O.table_key_u64(sh, b, z)
    keys = sorted(zip(hi.tolist(), lo.tolist()))
    spl = [keys[1000], keys[1000], keys[2500]]          # a repeated splitter leaves an empty range
    order, counts = O.key_partition(sh, b, z, [s[0] for s in spl], [s[1] for s in spl])
    assert counts.sum() == 4000 and counts[1] == 0
    d = [sum(1 for s in spl if s <= k) for k in zip(hi.tolist(), lo.tolist())]
    exp = sorted(range(4000), key=lambda i: (d[i], i))
    assert order.tolist() == exp


def _granges_worker(rank, world, port, q, dst=0):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geomesa_amd.ranges import RANGE_DTYPE
        from geomesa_amd.shard import gather_ranges
        nq = 3 + rank
        cnt = np.arange(nq) % 3 + rank
        off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        rr = np.zeros(int(off[-1]), RANGE_DTYPE)
        rr["lower"] = np.arange(len(rr)) + 1000 * rank
        rr["upper"] = rr["lower"] + 1
        rr["contained"] = rank
        g = gather_ranges(dist, off, rr, dst=dst)
        q.put((rank, g))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dst", [0, 1])
def test_gather_ranges(dst):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_granges_worker, args=(r, world, port, q, dst)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[1 - dst] is None
    off, rr = got[dst]
    c0, c1 = np.arange(3) % 3, np.arange(4) % 3 + 1
    assert off.tolist() == np.concatenate([[0], np.cumsum(np.concatenate([c0, c1]))]).tolist()
    assert rr["lower"].tolist() == list(range(c0.sum())) + [1000 + i for i in range(c1.sum())]
    assert rr["contained"].tolist() == [0] * c0.sum() + [1] * c1.sum()


def _grows_worker(rank, world, port, sizes, dst, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geomesa_amd.shard import gather_rows
        k = sizes[rank]
        ids = torch.arange(k, dtype=torch.int64) + 1000 * rank
        pl = torch.full((k,), rank, dtype=torch.int32)
        g = gather_rows(dist, [ids, pl], dst=dst)
        q.put((rank, None if g is None else (g[0].numpy(), g[1].numpy())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes,dst", [((5, 0, 3), 0), ((0, 4, 2), 0), ((2, 7, 0), 1), ((0, 0, 0), 2)])
def test_gather_rows_exact_sizes(sizes, dst):
    """gather_rows: rank order, exact per-rank counts (empty ranks included, also the destination),
    nothing on the other ranks (shard.py gather_rows)."""
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grows_worker, args=(r, world, port, sizes, dst, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert (got[r] is None) == (r != dst)
    ids, pl = got[dst]
    assert ids.tolist() == [1000 * r + i for r in range(world) for i in range(sizes[r])]
    assert pl.tolist() == [r for r in range(world) for _ in range(sizes[r])]
    assert ids.dtype == np.int64 and pl.dtype == np.int32


def _gcompact_worker(rank, world, port, sizes, n_polys, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geomesa_amd.shard import gather_pairs_compact
        k = sizes[rank]
        base = (3 << 32) + rank * ((1 << 32) + 17)      # each rank's first global row
        g = torch.Generator().manual_seed(rank)
        rows = torch.randint(0, 1 << 32, (k,), generator=g, dtype=torch.int64)
        if k:
            rows[0] = (1 << 32) - 1                      # the top of the u32 range (sign bit set on the wire)
        pl = torch.randint(0, n_polys, (k,), generator=g, dtype=torch.int64).to(torch.int32)
        if k:
            pl[-1] = n_polys - 1
        got, wire = gather_pairs_compact(dist, rows + base, pl, base, n_polys, dst=0)
        q.put((rank, (rows + base).numpy(), pl.numpy(), None if got is None else (got[0].numpy(), got[1].numpy()), wire))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes,n_polys", [((5, 0, 3000), 65536), ((0, 4, 2), 3200), ((100, 7, 0), 70000)])
def test_gather_pairs_compact_round_trip(sizes, n_polys):
    """The join's compact result gather (4-B shard-local rows + 2-B polygon ids on the wire, expanded on
    rank 0) delivers exactly the (int64 point id, int32 polygon id) pairs of the full gather, in rank
    order; past 65,536 polygons it falls back to the 12-B format."""
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gcompact_worker, args=(r, world, port, sizes, n_polys, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, ids, pl, g, wire = q.get(timeout=240)
        got[r] = (ids, pl, g, wire)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    pt, pp = got[0][2]
    assert pt.dtype == np.int64 and pp.dtype == np.int32
    assert np.array_equal(pt, np.concatenate([got[r][0] for r in range(world)]))
    assert np.array_equal(pp, np.concatenate([got[r][1] for r in range(world)]))
    per = 6 if n_polys <= 65536 else 12
    assert got[0][3] == [per * s for s in sizes]
    assert all(got[r][2] is None for r in range(1, world))
