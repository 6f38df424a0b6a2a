"""GPU tests of the multi-rank join plumbing: a built index exported and imported (what
shard.broadcast_index ships over RCCL), and a 2-process gloo run on the one GPU of the box where rank 0
builds the index, broadcasts it, and every rank joins its point shard."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_gpu_scan_join_ranges import _sorted_pairs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_index_export_import_same_pairs(gpu, oracle):
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(20, 10)
    ix = PolygonIndex(ps)
    lay, arrs = ix.export_arrays()
    ix2 = PolygonIndex.from_arrays(lay, arrs)
    del arrs
    assert ix2.stats() == ix.stats()
    px, py = synthetic_points(300_000, seed=3)
    a = _sorted_pairs(*ix.join(px, py))
    b = _sorted_pairs(*ix2.join(px, py))
    assert np.array_equal(a, b)
    poly = np.arange(len(px)) % ps.n_polys
    assert bool((ix.relate(poly, px, py) == ix2.relate(poly, px, py)).all())


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geomesa_amd import _lib
        from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
        from geomesa_amd.shard import broadcast_index, gather_rows, shard_bounds
        torch.cuda.set_device(0)
        ctx = _lib.context(0)
        ix = PolygonIndex(synthetic_counties(20, 10), ctx) if rank == 0 else None
        ix = broadcast_index(dist, ix, 0, ctx)
        n = 400_003
        px, py = synthetic_points(n, seed=12)
        lo, hi = shard_bounds(n, rank, world)
        pt, pl = ix.join(px[lo:hi], py[lo:hi], id_base=lo)
        g = gather_rows(dist, [pt.cpu(), pl.cpu()])
        if rank == 0:
            q.put(np.stack([g[0].numpy(), g[1].numpy().astype(np.int64)], 1))
    finally:
        dist.destroy_process_group()


def test_broadcast_index_sharded_join(gpu, oracle):
    from geomesa_amd.join import synthetic_counties, synthetic_points
    world = 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    px, py = synthetic_points(400_003, seed=12)
    opt, opl = oracle.OraclePolySet(*synthetic_counties(20, 10).to_arrays()).join(px, py, nthreads=16)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    got = got[np.lexsort((got[:, 1], got[:, 0]))]
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    assert np.array_equal(got, exp)


# ---------------------------------------------------------------- key-range partitioned table (configs[2])

def _table_points(n=600_001, seed=4):
    rng = np.random.default_rng(seed)
    x = rng.uniform(-180, 180, n)
    y = rng.uniform(-90, 90, n)
    t = rng.integers(1590969600000, 1590969600000 + 5 * 604800000, n)   # five weeks from 2020-06-01
    sh = (np.arange(n) * 2654435761 % 4).astype(np.uint8)               # a 4-way shard byte
    return x, y, t, sh


TABLE_QUERIES = [([(-10, 35, 30, 60)], [(1590969600000, 1591617600000)]),
                 ([(100, -40, 160, 0)], [(1591500000000, 1592900000000)]),
                 ([(-180, -90, 180, 90)], [(1590969600000, 1593000000000)]),
                 ([(0, 0, 0.5, 0.5)], [(1590969600000, 1594000000000)])]


def _table_worker(rank, world, port, sharded, idmode, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from geomesa_amd.keyspace import during
        from geomesa_amd.shard import gather_rows, shard_bounds
        from geomesa_amd.table import PartitionedZ3Table
        torch.cuda.set_device(0)
        x, y, t, sh = _table_points()
        lo, hi = shard_bounds(len(x), rank, world)
        ids = np.arange(lo, hi) if idmode == "ids" else lo   # a global-id column, or the first row's id
        tb = PartitionedZ3Table.from_points(dist, x[lo:hi], y[lo:hi], t[lo:hi], ids,
                                            shard=sh[lo:hi] if sharded else None, shards=4 if sharded else None,
                                            samples=256)
        res = [tb.n, tb.timing]
        for bxs, ts in TABLE_QUERIES:
            got, nm, ns, nr = tb.query(bxs, [during(a, b) for a, b in ts])
            g = gather_rows(dist, [got.cpu()])
            if rank == 0:
                res.append(np.sort(g[0].numpy()))
        q.put(res if rank == 0 else res[:2])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sharded,idmode,world", [(False, "ids", 2), (True, "ids", 2), (False, "base", 2),
                                                  (True, "base", 3)])
def test_partitioned_table_equals_oracle_scan(gpu, oracle, sharded, idmode, world):
    """Ranks sharing the box's GPU (gloo): each keys its unsorted rows, the ranks agree on splitters from
    key samples, one partition pass + one all-to-all per column + one sort per rank builds the slices,
    and each rank scans the query ranges clipped to its slice.  The gathered global ids equal the
    oracle's z3filter_scan (C restatement of Z3Filter.inBounds, Z3Filter.scala:26-62) over every row."""
    from geomesa_amd import filters as F
    from geomesa_amd.keyspace import Z3IndexKeySpace, during
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_table_worker, args=(r, world, port, sharded, idmode, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = max(got, key=len)
    sizes = sorted(g[0] for g in got)
    x, y, t, sh = _table_points()
    assert sum(sizes) == len(x) and sizes[0] > 0.8 * len(x) / world   # balanced key ranges
    for g in got:   # one sort per rank: the ingest's phases are a partition, an exchange and a sort
        assert set(g[1]) >= {"partition_ms", "exchange_ms", "sort_ms"} and sum(g[1]["received_rows"]) == g[0]
    ks = Z3IndexKeySpace()
    ob, oz, _ = oracle.z3_index_key_batch(x, y, t)
    for k, (bxs, ts) in enumerate(TABLE_QUERIES):
        v = ks.get_index_values(bxs, [during(a, b) for a, b in ts])
        om = oracle.z3filter_scan(F.serialize_to_bytes(F.Z3Filter.from_values(v)), ks.bin_ranges(v), ob, oz)
        exp = np.nonzero(om)[0]
        assert len(exp) > 0 or k == 3
        assert np.array_equal(full[2 + k], exp), k


def test_partitioned_table_single_slice(gpu):
    """pg None: one slice, no exchange; the query ids equal the plain table's."""
    from geomesa_amd.keyspace import during
    from geomesa_amd.table import PartitionedZ3Table, Z3Table
    x, y, t, sh = _table_points(200_001, seed=9)
    ids = np.arange(len(x)) + 1000
    pt = PartitionedZ3Table.from_points(None, x, y, t, ids, shard=sh, shards=4)
    tb = Z3Table.from_points(x, y, t, shard=sh)
    for bxs, ts in TABLE_QUERIES:
        got, nm, ns, nr = pt.query(bxs, [during(a, b) for a, b in ts])
        exp, _, _ = tb.query(bxs, [during(a, b) for a, b in ts])
        assert np.array_equal(np.sort(got.cpu().numpy()), np.sort(exp.cpu().numpy()) + 1000)
