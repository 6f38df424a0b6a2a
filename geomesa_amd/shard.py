"""Multi-GPU plumbing for the hot path: one process per GPU, points sharded by contiguous row range.

Every operation on the path is independent per point (Z3/Z2/XZ keys, filter scans, the
st_contains join against a replicated polygon set), so ranks shard the points and run with no
data-path collective ("weak" scaling).  The only exchanges are the polygon-set broadcast before a
join (the reference ships the smaller side of the join to every partition: GeoMesaJoinRelation /
RelationUtils.grid, geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91) and the scalar
max/sum reductions of the benchmark, plus the result gather: per-rank match counts, then the
ids / (point, polygon) pairs to one rank (gather_rows).  Works with both RCCL ("nccl", device
tensors) and gloo (CPU tensors, used by the multi-process tests).
"""
import numpy as np


def shard_bounds(n_total, rank, world):
    """Contiguous [lo, hi) rows of rank `rank` out of `world` (sizes differ by at most one)."""
    if world < 1 or not 0 <= rank < world or n_total < 0:
        raise ValueError("bad shard request: n=%d rank=%d world=%d" % (n_total, rank, world))
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _device_of(pg):
    return "cuda" if pg.get_backend() == "nccl" else "cpu"


def broadcast_polyset(pg, ps, src=0):
    """Broadcast a PolygonSet from rank `src`; other ranks pass ps=None and get the copy back."""
    import torch
    from .join import PolygonSet
    dev = _device_of(pg)
    arrs = ps.to_arrays() if pg.get_rank() == src else None
    sizes = torch.tensor([len(v) for v in arrs] if arrs else [0] * 5, dtype=torch.int64, device=dev)
    pg.broadcast(sizes, src)
    out = []
    for k, (sz, dt) in enumerate(zip(sizes.tolist(), [torch.int32] * 3 + [torch.float64] * 2)):
        t = torch.from_numpy(np.ascontiguousarray(arrs[k])).to(dev) if arrs else torch.empty(sz, dtype=dt, device=dev)
        pg.broadcast(t, src)
        out.append(t.cpu().numpy())
    return PolygonSet(*out)


def broadcast_index(pg, index, src=0, ctx=None):
    """Broadcast a built join index (join.PolygonIndex) from rank `src`: its device arrays go out over
    RCCL (xGMI) and every other rank imports them (gm_pip_index_import) -- no per-rank host rebuild.
    Other ranks pass index=None.  Over gloo the arrays travel through host memory."""
    import ctypes
    import torch
    from . import _lib
    from .join import PolygonIndex
    dev = _device_of(pg)
    nb = ctypes.sizeof(_lib.PipIndexLayout)
    if pg.get_rank() == src:
        lay, arrs = index.export_arrays()
        hdr = torch.frombuffer(bytearray(bytes(lay)), dtype=torch.uint8).to(dev)
    else:
        lay, arrs = None, None
        hdr = torch.zeros(nb, dtype=torch.uint8, device=dev)
    pg.broadcast(hdr, src)
    if pg.get_rank() != src:
        lay = _lib.PipIndexLayout.from_buffer_copy(bytes(hdr.cpu().numpy().tobytes()))
    out = []
    cuda = torch.device("cuda", (ctx or _lib.context()).device)
    for k in range(_lib.GM_PIP_INDEX_ARRAYS):
        size = max(int(lay.bytes[k]), 1)
        t = arrs[k].to(dev) if arrs is not None else torch.empty(size, dtype=torch.uint8, device=dev)
        pg.broadcast(t, src)
        out.append(t.to(cuda))
    if pg.get_rank() == src:
        return index
    return PolygonIndex.from_arrays(lay, out, ctx)


def all_reduce_scalar(pg, v, op="max"):
    """max / sum of one float over all ranks (identity without a process group)."""
    if pg is None:
        return float(v)
    import torch
    t = torch.tensor([float(v)], dtype=torch.float64, device=_device_of(pg))
    pg.all_reduce(t, op={"max": pg.ReduceOp.MAX, "sum": pg.ReduceOp.SUM}[op])
    return float(t.item())


def gather_rows(pg, cols, dst=0):
    """Gather variable-length per-rank result columns (1-D tensors of equal length per rank: ids,
    or point ids + polygon ids) to rank `dst`, in rank order.

    One all_gather of the per-rank counts (8 B each), then one gather of each column padded to the
    largest count: over RCCL a gather is a grouped send/recv, so rank `dst` receives from every
    peer at once over its own xGMI link (padding costs at most the imbalance between ranks).
    Returns the concatenated columns on `dst` and None elsewhere; with pg None, `cols`."""
    if pg is None:
        return list(cols)
    import torch
    dev = _device_of(pg)
    world = pg.get_world_size()
    n = torch.tensor([int(cols[0].numel())], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    pg.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    mx = max(counts)
    out = []
    for c in cols:
        buf = torch.zeros(mx, dtype=c.dtype, device=dev)
        buf[:c.numel()] = c.to(dev)
        parts = [torch.empty_like(buf) for _ in range(world)] if pg.get_rank() == dst else None
        pg.gather(buf, parts, dst=dst)
        out.append(torch.cat([p[:k] for p, k in zip(parts, counts)]) if pg.get_rank() == dst else None)
    return out if pg.get_rank() == dst else None


def merge_histograms(pg, counts, present, bin_lo, length=None):
    """Z3Histogram `+=` across ranks (utils/stats/Z3Histogram.scala:145-160): each rank's dense block of
    time-bin rows [bin_lo, bin_lo + rows) is placed into the union window and summed (counts) / OR'd
    (present) with two all-reduces over RCCL (gloo on CPU).  A rank with no histogram passes
    counts=None.  Returns (counts [rows, length], present [rows], bin_lo) of the merged binMap on every
    rank, or (None, None, None) when every rank is empty.

    The reference throws for histograms of different lengths; here every rank learns the min and the
    max length from scalar all-reduces first and raises together, before any tensor collective (one
    rank raising alone would leave the others waiting in the all-reduce).  With pg None the input is
    returned as it is."""
    import torch
    if pg is None:
        if counts is None:
            return None, None, None
        return counts, present, bin_lo
    dev = _device_of(pg)
    big = float(1 << 20)
    have = counts is not None
    lo = float(bin_lo) if have else big
    hi = float(bin_lo + counts.shape[0] - 1) if have else -big
    ln = float(counts.shape[1]) if have else float(length or 0)
    lo, hi = -all_reduce_scalar(pg, -lo, "max"), all_reduce_scalar(pg, hi, "max")
    len_max = all_reduce_scalar(pg, ln if have else -big, "max")
    len_min = -all_reduce_scalar(pg, -ln if have else -big, "max")
    if hi < lo:
        return None, None, None
    if len_max != len_min:
        raise NotImplementedError("Can only add z3 histograms with the same length")
    length = int(len_max)
    lo, hi = int(lo), int(hi)
    rows = hi - lo + 1
    c = torch.zeros((rows, length), dtype=torch.int64, device=dev)
    p = torch.zeros(rows, dtype=torch.int64, device=dev)   # int64: gloo has no uint8 MAX on every build
    if have:
        off = bin_lo - lo
        c[off:off + counts.shape[0]] = counts.to(dev) * (present.to(dev) != 0).to(torch.int64).unsqueeze(1)
        p[off:off + counts.shape[0]] = present.to(dev).to(torch.int64)
    pg.all_reduce(c, op=pg.ReduceOp.SUM)
    pg.all_reduce(p, op=pg.ReduceOp.MAX)
    return c, (p != 0).to(torch.uint8), lo
