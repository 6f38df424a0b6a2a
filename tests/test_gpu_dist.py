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
    for mode in ("direct", "split", "partitioned"):
        a = _sorted_pairs(*ix.join(px, py, mode=mode))
        b = _sorted_pairs(*ix2.join(px, py, mode=mode))
        assert np.array_equal(a, b), mode
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
