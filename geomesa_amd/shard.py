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


def broadcast_index(pg, index, src=0, ctx=None, reimport=False):
    """Broadcast a built join index (join.PolygonIndex) from rank `src`: its device arrays go out over
    RCCL (xGMI) and every other rank imports them (gm_pip_index_import) -- no per-rank host rebuild.
    Other ranks pass index=None.  Over gloo the arrays travel through host memory.  reimport=True makes
    `src` import what it broadcast too (a test hook: at world 1 it runs the receiving side)."""
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
    if pg.get_rank() == src and not reimport:
        return index
    return PolygonIndex.from_arrays(lay, out, ctx)


def all_reduce_scalar(pg, v, op="max"):
    """max / min / sum of one float over all ranks (identity without a process group)."""
    if pg is None:
        return float(v)
    import torch
    t = torch.tensor([float(v)], dtype=torch.float64, device=_device_of(pg))
    pg.all_reduce(t, op={"max": pg.ReduceOp.MAX, "min": pg.ReduceOp.MIN, "sum": pg.ReduceOp.SUM}[op])
    return float(t.item())


def gather_rows(pg, cols, dst=0, loopback=False):
    """Gather variable-length per-rank result columns (1-D tensors of equal length per rank: ids,
    or point ids + polygon ids) to rank `dst`, in rank order.

    One all_gather of the per-rank counts (8 B each); then rank `dst` allocates each column once at
    its exact total and receives every peer's rows straight into that peer's slice (point-to-point,
    batched: over RCCL a group of sends / receives, so `dst` takes every peer's rows at once over its
    own xGMI link), and copies its own rows in.  No padding and no concatenation copy: rank `dst`
    holds the result and nothing else.  Returns the columns on `dst` and None elsewhere; with pg None,
    `cols`.  loopback=True moves `dst`'s own rows through the same send / receive group instead of a
    copy (a test hook: at world 1 it is how the RCCL point-to-point path runs on a one-GPU box)."""
    if pg is None:
        return list(cols)
    import torch
    dev = _device_of(pg)
    world, rank = pg.get_world_size(), pg.get_rank()
    n = torch.tensor([int(cols[0].numel())], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    pg.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    out, ops, keep = [], [], []
    for c in cols:
        if rank == dst:
            o = torch.empty(offs[-1], dtype=c.dtype, device=dev)
            if loopback and counts[dst] > 0:
                src = c.to(dev).contiguous()
                keep.append(src)
                ops.append(pg.P2POp(pg.isend, src, dst))
                ops.append(pg.P2POp(pg.irecv, o[offs[dst]:offs[dst + 1]], dst))
            else:
                o[offs[dst]:offs[dst + 1]] = c.to(dev)
            for r in range(world):
                if r != dst and counts[r] > 0:
                    ops.append(pg.P2POp(pg.irecv, o[offs[r]:offs[r + 1]], r))
            out.append(o)
        elif counts[rank] > 0:
            src = c.to(dev).contiguous()
            keep.append(src)
            ops.append(pg.P2POp(pg.isend, src, dst))
    if ops:
        for req in pg.batch_isend_irecv(ops):
            req.wait()
    return out if rank == dst else None


# xGMI on MI355X: 7 point-to-point links per GPU, ~153 GB/s each (MI355X_MICROARCH.md); rank dst takes
# every peer's rows at once, each over its own link, so a gather costs its largest peer's bytes / link
XGMI_LINK_GBS = 153.0


def gather_pairs_compact(pg, pt_ids, pl_ids, id_base, n_polys, dst=0, loopback=False):
    """The join's result gather (GeoMesaJoinRelation.scala:41-91 leaves the pairs in the RDD's
    partitions; here they come to rank `dst`) in a compact wire format: each rank's pairs travel as a
    4-B shard-local row (point id - the rank's id_base) and a 2-B polygon id -- 6 B per pair instead of
    12 -- and rank `dst` expands them to (int64 point id, int32 polygon id) in rank order, exactly the
    pairs gather_rows would deliver.  The full 12-B format is used when some rank's rows do not fit 32
    bits or there are more than 65,536 polygons.  Returns ((pt, pl), wire_bytes_per_rank) on `dst` and
    (None, wire_bytes_per_rank) elsewhere; with pg None, ((pt_ids, pl_ids), [12 * n])."""
    import torch
    n = int(pt_ids.numel())
    if pg is None:
        return (pt_ids, pl_ids), [12 * n]
    dev = _device_of(pg)
    world, rank = pg.get_world_size(), pg.get_rank()
    span = int((pt_ids.max() - id_base).item()) + 1 if n else 0
    lo_ok = n == 0 or int(pt_ids.min().item()) >= id_base
    mine = torch.tensor([n, int(id_base), int(span <= (1 << 32) and lo_ok)], dtype=torch.int64, device=dev)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    pg.all_gather(allv, mine)
    counts = [int(v[0].item()) for v in allv]
    bases = [int(v[1].item()) for v in allv]
    compact = n_polys <= (1 << 16) and all(int(v[2].item()) for v in allv)
    if not compact:
        g = gather_rows(pg, [pt_ids, pl_ids], dst, loopback)
        return (tuple(g) if g is not None else None), [12 * c for c in counts]
    # one byte buffer per rank -- [4-B rows | 2-B polygons | pad to 8 B] -- so a peer's pairs are one
    # point-to-point message (RCCL moves no int16 tensors) and every segment stays 8-B aligned on dst
    rows = (pt_ids - id_base).to(torch.int64)
    rows = torch.where(rows >= (1 << 31), rows - (1 << 32), rows).to(torch.int32)    # the u32 bit pattern
    polys = torch.where(pl_ids >= (1 << 15), pl_ids - (1 << 16), pl_ids).to(torch.int16)   # the u16 bit pattern
    seg = lambda c: (6 * c + 7) // 8 * 8   # noqa: E731
    buf = torch.zeros(seg(n), dtype=torch.uint8, device=pt_ids.device)
    buf[:4 * n] = rows.view(torch.uint8)
    buf[4 * n:6 * n] = polys.view(torch.uint8)
    g = gather_rows(pg, [buf], dst, loopback)
    if rank != dst:
        return None, [6 * c for c in counts]
    out, o = g[0], 0
    rs, ps = [], []
    for c in counts:
        part = out[o:o + seg(c)]
        rs.append(part[:4 * c].view(torch.int32))
        ps.append(part[4 * c:6 * c].view(torch.int16))
        o += seg(c)
    r, p = torch.cat(rs), torch.cat(ps)
    base = torch.repeat_interleave(torch.tensor(bases, dtype=torch.int64, device=dev),
                                   torch.tensor(counts, dtype=torch.int64, device=dev))
    pt = (r.to(torch.int64) & 0xFFFFFFFF) + base
    pl = p.to(torch.int32) & 0xFFFF
    return (pt, pl), [6 * c for c in counts]


def gather_estimate_ms(wire_bytes, dst=0, hbm_gbs=5000.0):
    """The gather's model time: the largest peer's bytes over one xGMI link (the peers send at once,
    each on its own link), against rank dst's HBM writing every received byte; the larger of the two."""
    peers = [b for r, b in enumerate(wire_bytes) if r != dst]
    link = max(peers) / (XGMI_LINK_GBS * 1e9) * 1e3 if peers else 0.0
    hbm = sum(peers) / (hbm_gbs * 1e9) * 1e3
    return max(link, hbm)


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


# ---------------------------------------------------------------- key-range partitioned table
# configs[2]: the table's rows are split into `world` contiguous key ranges, one per GPU, the way a
# sorted store splits a table into tablets / regions; a query's scan ranges are clipped to each
# slice (what the client's range binning does per tablet) and every GPU scans only its part.
# Keys compare as the row bytes do: [shard][bin BE16][z BE64], unsigned.  The ingest (every rank's
# unsorted rows -> sample_keys -> choose_splitters -> partition_rows -> exchange_partitioned -> one
# gm_sort_keys of the received slice) carries them as (key_hi = shard << 16 | bin as u16, key_lo = z)
# uint64 pairs; the slice bounds and range clipping below use two int64 values of the same
# lexicographic order:
#   hi = shard << 16 | bin as unsigned short       lo = z with the sign bit flipped

_SIGN = -(1 << 63)


def table_key(shard, bin, z):
    """(hi, lo) int64 key columns (torch) of (shard uint8 or None, bin int16, z int64) columns."""
    import torch
    hi = bin.to(torch.int64) & 0xffff
    if shard is not None:
        hi = hi | (shard.to(torch.int64) << 16)
    return hi, z.to(torch.int64) ^ _SIGN


def sample_keys(ctx, shard, bin, z, samples=1024):
    """`samples` keys of one rank's UNSORTED key columns (evenly spaced rows), gm_key_sample: (key_hi,
    key_lo) uint64 numpy arrays, key_hi = shard << 16 | bin as u16, key_lo = z -- the row-key byte order."""
    from . import _lib
    n = int(z.numel())
    k = min(int(samples), 65536) if n else 0
    hi, lo = np.zeros(k, np.uint64), np.zeros(k, np.uint64)
    if k:
        _lib.check(ctx.lib.gm_key_sample(ctx.handle, _lib.ptr(shard), _lib.ptr(bin), _lib.ptr(z), n, k,
                                         hi.ctypes.data, lo.ctypes.data), "gm_key_sample")
    return hi, lo


def choose_splitters(pg, s_hi, s_lo, n, samples=1024):
    """world - 1 splitter keys (key_hi, key_lo uint64 numpy arrays, identical on every rank) from every
    rank's key sample (sample_keys of its n rows, at most `samples` keys), each sample weighted by the
    rows it stands for, so each key range holds about 1/world of all rows.  One all_gather of the
    samples (host planning, like a client's split planning; no per-splitter device sync)."""
    import torch
    world = pg.get_world_size() if pg is not None else 1
    if world == 1:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint64)
    k = len(s_hi)
    cap = max(1, min(int(samples), 65536))
    if k > cap:
        raise ValueError("%d samples for a cap of %d" % (k, cap))
    dev = _device_of(pg)
    s = torch.zeros((cap, 4), dtype=torch.int64)
    if k:
        s[:k, 0] = torch.from_numpy(np.ascontiguousarray(s_hi, np.uint64).view(np.int64))
        s[:k, 1] = torch.from_numpy(np.ascontiguousarray(s_lo, np.uint64).view(np.int64))
        s[:k, 2] = int(n)
        s[:k, 3] = k
    parts = [torch.zeros_like(s).to(dev) for _ in range(world)]
    pg.all_gather(parts, s.to(dev))
    allv = torch.cat([p.cpu() for p in parts]).numpy()
    keep = allv[:, 3] > 0
    allv = allv[keep]
    if len(allv) == 0:
        return np.zeros(world - 1, np.uint64), np.zeros(world - 1, np.uint64)
    w = allv[:, 2].astype(np.float64) / allv[:, 3]       # rows each sample stands for
    hi, lo = allv[:, 0].view(np.uint64), allv[:, 1].view(np.uint64)
    order = np.lexsort((lo, hi))
    cw = np.cumsum(w[order])
    idx = np.minimum(np.searchsorted(cw, cw[-1] * np.arange(1, world) / world, side="left"), len(allv) - 1)
    return hi[order][idx].copy(), lo[order][idx].copy()


def partition_rows(ctx, shard, bin, z, sp_hi, sp_lo, ids=None, id_base=0, rows=False):
    """The rank's rows grouped by destination key range (gm_key_partition: one count read, a device scan,
    one scatter read; stable within a destination).  Returns ([shard?, bin, z, src], counts): device
    columns in destination order -- src = ids[row] (ids given, int64), the input row as int32 (rows=True:
    4 B on the wire instead of 8) or id_base + row (int64) -- and the per-destination row counts."""
    import torch
    from . import _lib
    n = int(z.numel())
    nd = len(sp_hi) + 1
    dev = z.device
    sh_o = torch.empty(n, dtype=torch.uint8, device=dev) if shard is not None else None
    b_o, z_o = torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int64, device=dev)
    src = torch.empty(n, dtype=torch.int32 if rows else torch.int64, device=dev)
    counts = np.zeros(nd, np.int64)
    hi = np.ascontiguousarray(sp_hi, np.uint64)
    lo = np.ascontiguousarray(sp_lo, np.uint64)
    _lib.check(ctx.lib.gm_key_partition(ctx.handle, _lib.ptr(shard), _lib.ptr(bin), _lib.ptr(z), n,
                                        hi.ctypes.data if len(hi) else None, lo.ctypes.data if len(lo) else None,
                                        len(hi), _lib.ptr(ids), int(id_base), _lib.ptr(sh_o), _lib.ptr(b_o),
                                        _lib.ptr(z_o), None if rows else _lib.ptr(src), _lib.ptr(src) if rows else None,
                                        counts.ctypes.data), "gm_key_partition")
    cols = ([sh_o] if shard is not None else []) + [b_o, z_o, src]
    return cols, counts.tolist()


def exchange_partitioned(pg, cols, send):
    """All-to-all of destination-grouped columns (partition_rows): rank r receives every peer's
    destination-r slice of each column, in rank order.  One all_to_all of the counts, then one per column
    (each column moved as bytes, so any dtype travels: RCCL has no int16); over RCCL every xGMI link
    carries its peer's slice at once.  Returns (received columns, received counts per source rank)."""
    import torch
    world = pg.get_world_size()
    dev = _device_of(pg)
    sc = torch.tensor([int(v) for v in send], dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    pg.all_to_all_single(rc, sc)
    recv = [int(v) for v in rc.cpu().tolist()]
    out = []
    def as_bytes(t):   # (an empty tensor has no byte view)
        return t.contiguous().view(torch.uint8) if t.numel() else torch.empty(0, dtype=torch.uint8, device=t.device)
    for c in cols:
        k = c.element_size()
        src = as_bytes(c).to(dev)
        o = torch.empty(sum(recv) * k, dtype=torch.uint8, device=dev)
        pg.all_to_all_single(o, src, [r * k for r in recv], [int(s) * k for s in send])
        del src
        out.append(o.to(c.device).view(c.dtype) if o.numel() else torch.empty(0, dtype=c.dtype, device=c.device))
    return out, recv


def clip_key_ranges(ranges, kmin, kmax):
    """Clip gm_key_range rows (numpy KEY_RANGE_DTYPE array) to the key slice [kmin, kmax] (each an
    (hi, lo) key pair, inclusive): ranges outside are dropped, the rest narrowed.  A range lies in
    one shard and the slice bounds are keys of that ordering, so a clipped range stays in its shard."""
    r = np.asarray(ranges)
    if kmin is None or len(r) == 0:
        return r[:0].copy()
    sh = r["shard"].astype(np.int64) << 16
    l_hi = sh | (r["bin_lo"].astype(np.int64) & 0xffff)
    h_hi = sh | (r["bin_hi"].astype(np.int64) & 0xffff)
    l_lo = r["z_lo"] ^ np.int64(_SIGN)
    h_lo = r["z_hi"] ^ np.int64(_SIGN)

    def less(ah, al, bh, bl):
        return (ah < bh) | ((ah == bh) & (al < bl))
    # new lower = max(L, kmin), new upper = min(H, kmax)
    up = less(l_hi, l_lo, kmin[0], kmin[1])
    n_hi, n_lo = np.where(up, kmin[0], l_hi), np.where(up, kmin[1], l_lo)
    dn = less(kmax[0], kmax[1], h_hi, h_lo)
    x_hi, x_lo = np.where(dn, kmax[0], h_hi), np.where(dn, kmax[1], h_lo)
    keep = ~less(x_hi, x_lo, n_hi, n_lo)
    out = r[keep].copy()

    def s16(v):
        return (((v & 0xffff) ^ 0x8000) - 0x8000).astype(np.int16)
    out["bin_lo"], out["z_lo"] = s16(n_hi[keep]), n_lo[keep] ^ np.int64(_SIGN)
    out["bin_hi"], out["z_hi"] = s16(x_hi[keep]), x_lo[keep] ^ np.int64(_SIGN)
    return out


def gather_ranges(pg, out_off, ranges, dst=0):
    """Gather per-rank batched-ranges results (out_off [nq_r + 1] int64, ranges numpy RANGE_DTYPE) of
    contiguous query shards to rank `dst`: (out_off, ranges) over all queries in rank order there,
    None elsewhere; with pg None the input."""
    if pg is None:
        return out_off, ranges
    import torch
    from .ranges import RANGE_DTYPE
    cnt = torch.from_numpy(np.diff(np.asarray(out_off, np.int64)))
    rr = torch.from_numpy(np.ascontiguousarray(ranges).view(np.int64).reshape(-1).copy())
    g = gather_rows(pg, [cnt], dst=dst)
    gr = gather_rows(pg, [rr], dst=dst)
    if g is None:
        return None
    offs = np.concatenate([[0], np.cumsum(g[0].cpu().numpy())]).astype(np.int64)
    return offs, gr[0].cpu().numpy().view(RANGE_DTYPE)
