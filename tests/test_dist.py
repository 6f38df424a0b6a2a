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
