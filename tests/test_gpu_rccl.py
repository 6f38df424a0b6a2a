"""The RCCL ("nccl" backend) branches of the multi-GPU plumbing, run at world size 1 on the box's one
GPU.  Every other multi-rank test uses gloo; these run the device-tensor code paths that only the
8-GPU scaling run would otherwise reach first: the index broadcast and its import
(shard.broadcast_index), the exact-size point-to-point gather (shard.gather_rows, batch_isend_irecv
with P2POp), the key-range partition + per-column all_to_all_single with splits (shard.exchange_partitioned), the scalar and
histogram all-reduces, the ranges gather, and bench.py itself under torch.distributed.run with one
rank.  With one rank the collectives degenerate (a broadcast or all-to-all to oneself), so these
tests check plumbing -- arguments, devices, dtypes, P2POp construction -- not scaling.  They replace
the Spark shuffles of GeoMesaJoinRelation.scala:42 and RelationUtils.scala:30-33."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_worker(port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    res = {}
    try:
        from geomesa_amd import _lib
        from geomesa_amd import shard as S
        from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
        from geomesa_amd.ranges import RANGE_DTYPE
        res["backend"] = dist.get_backend()
        ctx = _lib.context(0)
        ix = PolygonIndex(synthetic_counties(20, 10), ctx)
        # the index broadcast over RCCL (device tensors), then imported from the received arrays
        ix2 = S.broadcast_index(dist, ix, 0, ctx, reimport=True)
        res["reimported"] = ix2 is not ix
        px, py = synthetic_points(200_003, seed=31)
        pt, pl = ix.join(px, py, id_base=5)
        pt2, pl2 = ix2.join(px, py, id_base=5)
        key = lambda a, b: np.sort(a.cpu().numpy() * 4096 + b.cpu().numpy())   # noqa: E731
        res["broadcast_pairs_equal"] = bool(np.array_equal(key(pt, pl), key(pt2, pl2)))
        res["pairs"] = int(pt.numel())
        # the exact-size gather: counts all_gather, then the rows through batch_isend_irecv (loopback)
        g = S.gather_rows(dist, [pt, pl], loopback=True)
        res["gather_equal"] = bool(torch.equal(g[0], pt) and torch.equal(g[1], pl))
        res["gather_device"] = str(g[0].device)
        g0 = S.gather_rows(dist, [pt[:0]], loopback=True)   # an empty rank: no point-to-point op
        res["gather_empty"] = int(g0[0].numel())
        # the compact wire format (4-B rows + 2-B polygons through the same P2P group), expanded on rank 0
        (ct, cl), wire = S.gather_pairs_compact(dist, pt, pl, 5, ix.polyset.n_polys, loopback=True)
        res["compact_equal"] = bool(torch.equal(ct, pt) and torch.equal(cl, pl) and ct.dtype == torch.int64 and
                                    cl.dtype == torch.int32)
        res["compact_wire"] = wire == [6 * int(pt.numel())]
        # the key-range ingest: key sample, splitters, the partition kernel and the per-column
        # all_to_all_single (bytes, with splits) of the destination runs, over RCCL device tensors
        z = torch.arange(1000, dtype=torch.int64, device="cuda") * 7919 % 1000
        b = (torch.arange(1000, device="cuda") % 5).to(torch.int16)
        shc = (torch.arange(1000, device="cuda") % 3).to(torch.uint8)
        s_hi, s_lo = S.sample_keys(ctx, shc, b, z, 64)
        sp = S.choose_splitters(dist, s_hi, s_lo, 1000, 64)
        cols, send = S.partition_rows(ctx, shc, b, z, *sp, id_base=10, rows=True)
        got, recv = S.exchange_partitioned(dist, cols, send)
        res["exchange_equal"] = bool(len(sp[0]) == 0 and send == [1000] and recv == [1000] and
                                     all(torch.equal(g, c) for g, c in zip(got, cols)) and
                                     got[0].device.type == "cuda" and got[1].dtype == torch.int16)
        res["exchange_world1"] = bool(torch.equal(got[3].to(torch.int64), torch.arange(1000, device="cuda")))
        # scalar and histogram all-reduces
        res["max"] = S.all_reduce_scalar(dist, 3.5, "max")
        res["sum"] = S.all_reduce_scalar(dist, 2.0, "sum")
        counts = torch.arange(12, dtype=torch.int64, device="cuda").reshape(3, 4)
        present = torch.tensor([1, 0, 1], dtype=torch.uint8, device="cuda")
        c, p, blo = S.merge_histograms(dist, counts, present, 7)
        res["hist_ok"] = bool(blo == 7 and torch.equal(p, present) and
                              torch.equal(c, counts * present.to(torch.int64).unsqueeze(1)))
        # the batched-ranges gather (offsets + ranges of the rank's queries)
        rr = np.zeros(5, RANGE_DTYPE)
        rr["lower"] = np.arange(5)
        rr["upper"] = np.arange(5) + 100
        rr["contained"] = [1, 0, 1, 0, 1]
        go, gr = S.gather_ranges(dist, np.array([0, 2, 5], np.int64), rr)
        res["ranges_equal"] = bool(np.array_equal(go, [0, 2, 5]) and np.array_equal(gr["upper"], rr["upper"]) and
                                   np.array_equal(gr["contained"], rr["contained"]))
        torch.cuda.synchronize()
    except Exception as e:   # noqa: BLE001 -- reported to the parent
        res["error"] = repr(e)
    finally:
        dist.destroy_process_group()
    q.put(res)


def test_shard_plumbing_over_rccl_world1(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["reimported"] and res["broadcast_pairs_equal"] and res["pairs"] > 0
    assert res["gather_equal"] and res["gather_device"].startswith("cuda") and res["gather_empty"] == 0
    assert res["compact_equal"] and res["compact_wire"]
    assert res["exchange_equal"] and res["exchange_world1"]
    assert res["max"] == 3.5 and res["sum"] == 2.0 and res["hist_ok"]
    assert res["ranges_equal"]


def test_bench_under_torchrun_world1(gpu):
    """bench.py under torch.distributed.run with one rank: Dist initialises the "nccl" group (every
    RCCL branch of the bench runs: index broadcast, pair gather, key-range table, ranges gather,
    max-over-ranks timing) at reduced sizes, and prints its one JSON line."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--join-steps", "1", "--points", "8000000",
           "--join-points", "4000000", "--table-rows", "2000000", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["pip_join"]["matches"] > 0
    detail = json.loads([ln for ln in r.stderr.splitlines() if ln.startswith("BENCH_DETAIL ")][-1][13:])
    pj = detail["pip_join"]
    assert pj["gather"].get("pairs_on_rank0") == pj["matches"], pj["gather"]
    assert pj["gather"].get("pairs_on_rank0_compact") == pj["matches"], pj["gather"]
    tq = detail["extra"]["table_query"]
    assert tq["parity"]["ids_equal"], tq["parity"]
