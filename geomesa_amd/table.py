"""A Z3 index table resident in HBM: ingest (keys -> table order) and seek-and-filter queries.

Mirrors the write and read sides of a GeoMesa Z3 index over a sorted key-value store:
  * ingest  -- Z3IndexKeySpace.toIndexKey (geomesa-index-api/.../index/z3/Z3IndexKeySpace.scala:63-95)
               for every feature, rows kept in key byte order by the store.  Here: gm_z3_index_key
               (bin, z columns), then gm_sort_keys into table order (the store's sort);
  * query   -- getIndexValues / getRanges / getRangeBytes (:97-238) plan the scan ranges, the
               store seeks each range and RowFilterIterator runs the Z3Filter on every row inside
               (geomesa-accumulo-iterators/.../RowFilterIterator.scala:52-66).  Here: ranges from
               the batched GPU ZN.zranges, then gm_key_range_scan (binary-searched row intervals +
               Z3Filter mask + ordered compaction).

The shard byte (ShardStrategy.scala:75-80: shards(feature.idHash % n)) is a column the caller
supplies; feature ids stay with the caller (results are input row indices).
"""
import ctypes

import numpy as np

from . import _lib
from . import filters as F
from ._lib import check, ptr
from .keyspace import Z3IndexKeySpace

_ALL64 = -1  # 0xFFFF... as int64


def key_ranges(scan_ranges, shards=None):
    """getRangeBytes (Z3IndexKeySpace.scala:196-238) as gm_key_range rows (numpy KEY_RANGE_DTYPE): one
    per scan range and shard.  scan_ranges are Z3IndexKeySpace.get_ranges tuples."""
    k = len(scan_ranges)
    zl, zh = np.zeros(k, np.int64), np.full(k, _ALL64, np.int64)
    bl, bh = np.zeros(k, np.int16), np.full(k, -1, np.int16)
    for i, (kind, lo, hi) in enumerate(scan_ranges):
        if kind == "bounded":
            zl[i], zh[i], bl[i], bh[i] = lo[1], hi[1], lo[0], hi[0]
        elif kind == "lower":
            zl[i], bl[i] = lo[1], lo[0]
        elif kind == "upper":
            zh[i], bh[i] = hi[1], hi[0]
    ns = shards if shards else 1
    arr = np.zeros(k * ns, _lib.KEY_RANGE_DTYPE)   # range-major, then shard (getRangeBytes order)
    arr["z_lo"], arr["z_hi"] = np.repeat(zl, ns), np.repeat(zh, ns)
    arr["bin_lo"], arr["bin_hi"] = np.repeat(bl, ns), np.repeat(bh, ns)
    arr["shard"] = np.tile(np.arange(ns, dtype=np.uint8), k)
    return arr, len(arr)


class Z3Table:
    """Sorted (shard, bin, z) key columns of one GPU's slice of a Z3 index table."""

    def __init__(self, bins, z, shard=None, period="week"):
        import torch
        from .curve import _dev_col
        self.ks = Z3IndexKeySpace(period)
        self.ctx = _lib.context()
        bins, z = _dev_col(bins, torch.int16), _dev_col(z, torch.int64)
        self.n = z.numel()
        dev = z.device
        self.bin = torch.empty_like(bins)
        self.z = torch.empty_like(z)
        self.perm = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.shards = None
        self.shard = None
        sh_in = None
        if shard is not None:
            sh_in = torch.as_tensor(np.asarray(shard, np.uint8) if not isinstance(shard, torch.Tensor) else shard,
                                    dtype=torch.uint8).to(dev).contiguous()
            self.shard = torch.empty_like(sh_in)
            self.shards = int(sh_in.max().item()) + 1 if self.n else 1
        check(self.ctx.lib.gm_sort_keys(self.ctx.handle, ptr(sh_in), ptr(bins), ptr(z), self.n, ptr(self.shard),
                                        ptr(self.bin), ptr(self.z), ptr(self.perm)), "gm_sort_keys")

    @classmethod
    def from_points(cls, x, y, t_ms, shard=None, period="week", lenient=False):
        ks = Z3IndexKeySpace(period)
        bins, z = ks.sfc.index_keys(x, y, t_ms, lenient=lenient)
        return cls(bins, z, shard, period)

    def key_bytes(self):
        """The table's row-key prefixes in table order, (n, 10|11) uint8 (gm_z3_key_bytes)."""
        import torch
        klen = 11 if self.shard is not None else 10
        out = torch.empty((self.n, klen), dtype=torch.uint8, device=self.z.device)
        check(self.ctx.lib.gm_z3_key_bytes(self.ctx.handle, ptr(self.shard), ptr(self.bin), ptr(self.z), self.n,
                                           ptr(out)), "gm_z3_key_bytes")
        return out

    def scan(self, scan_ranges, z3filter=None, map_rows=True, ids_cap=None):
        """Rows in any scan range that pass `z3filter` (a Z3Filter, its bytes, or None).

        Returns (ids tensor, n_match, n_scanned); ids are input rows (map_rows) or table rows."""
        arr, _ = key_ranges(scan_ranges, self.shards)
        return self.scan_key_ranges(arr, z3filter, map_rows, ids_cap)

    def scan_key_ranges(self, arr, z3filter=None, map_rows=True, ids_cap=None):
        """scan() over gm_key_range rows (numpy KEY_RANGE_DTYPE), e.g. ranges clipped to a slice."""
        import torch
        arr = np.ascontiguousarray(arr, _lib.KEY_RANGE_DTYPE)
        fb = None
        if z3filter is not None:
            fb = F.serialize_to_bytes(z3filter) if not isinstance(z3filter, (bytes, bytearray)) else bytes(z3filter)
        fbuf = (ctypes.c_uint8 * len(fb)).from_buffer_copy(fb) if fb else None
        cap = self.n if ids_cap is None else ids_cap
        ids = torch.empty(max(cap, 1), dtype=torch.int64, device=self.z.device)
        nm, ns = ctypes.c_int64(), ctypes.c_int64()
        rc = self.ctx.lib.gm_key_range_scan(self.ctx.handle, ptr(self.shard), ptr(self.bin), ptr(self.z), self.n,
                                            arr.ctypes.data if len(arr) else None, len(arr), fbuf,
                                            len(fb) if fb else 0, ptr(self.perm) if map_rows else None,
                                            ptr(ids), cap, ctypes.byref(nm), ctypes.byref(ns))
        if rc != _lib.GM_E_CAPACITY:
            check(rc, "gm_key_range_scan")
        return ids[:min(nm.value, cap)], nm.value, ns.value

    def query(self, bboxes=None, intervals=None, target=2000):
        """bbox + during query through the index (loose bbox, the default: Z3Filter only)."""
        v = self.ks.get_index_values(bboxes, intervals)
        if v.disjoint:
            import torch
            return torch.zeros(0, dtype=torch.int64, device=self.z.device), 0, 0
        sr = self.ks.get_ranges(v, target=target)
        return self.scan(sr, F.Z3Filter.from_values(v))


class PartitionedZ3Table:
    """configs[2]: a Z3 table range-partitioned over the GPUs of a process group, one slice per rank.

    Every rank starts from its own UNSORTED key columns (any split).  The ranks sample keys
    (gm_key_sample), agree on world - 1 splitter keys (one all_gather, host planning), and each rank
    writes its rows grouped by destination key range in one partition pass (gm_key_partition); one
    all-to-all per column moves every row to the rank owning its key range, which sorts what it
    received once (gm_sort_keys) -- one sort per rank, no sort before the exchange.  Afterwards rank r
    holds the rows of keys [splitter r-1, splitter r) in table order -- a sorted store's table split into
    tablets / regions (the shard prefix of ShardStrategy.scala:75-80 stays the key's first byte).  A
    query's scan ranges (getRangeBytes, Z3IndexKeySpace.scala:196-238) are clipped to the slice's first
    and last key (the per-tablet range binning of a batch scanner) and each rank scans only those; the
    ids that come back are global row ids, so the union over ranks equals the scan of one unpartitioned
    table.  The slice keeps each received row's source beside the table's permutation, so a scan maps
    only its matches to ids.  `ids` is either a column of global ids (8 B per row on the wire) or one
    int, the id of the rank's first row (ids = ids + row: 4-B rows on the wire, mapped back through the
    senders' bases).  pg None = a single unpartitioned slice.  `timing` holds the ingest's phases (ms,
    HIP events on the context stream)."""

    def __init__(self, pg, bins, z, ids, shard=None, shards=None, period="week", samples=1024):
        import torch
        from . import shard as S
        from .curve import _dev_col
        self.pg = pg
        sharded = shard is not None
        self.timing = {}
        self._recv_end, self._id_base = None, 0
        compact = isinstance(ids, (int, np.integer))
        if pg is None or pg.get_world_size() == 1:   # one slice: the local table is the table
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            local = Z3Table(bins, z, shard, period)
            ev[1].record()
            self.table, self.splitters = local, (np.zeros(0, np.uint64), np.zeros(0, np.uint64))
            if sharded and shards:
                self.table.shards = int(shards)
            dev = local.z.device
            self._recv_end, self._id_base = None, int(ids) if compact else 0
            self.src_ids = None if compact else torch.as_tensor(ids).to(dev, torch.int64)
            self.n = local.n
            ev[1].synchronize()
            self.timing = {"sort_ms": ev[0].elapsed_time(ev[1])}
            self._bounds()
            return
        ctx = _lib.context()
        bins, z = _dev_col(bins, torch.int16), _dev_col(z, torch.int64)
        dev = z.device
        sh_in = None
        if sharded:
            sh_in = torch.as_tensor(np.asarray(shard, np.uint8) if not isinstance(shard, torch.Tensor) else shard,
                                    dtype=torch.uint8).to(dev).contiguous()
        id_col = None if compact else torch.as_tensor(ids).to(dev, torch.int64).contiguous()
        n = int(z.numel())
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        s_hi, s_lo = S.sample_keys(ctx, sh_in, bins, z, samples)
        self.splitters = S.choose_splitters(pg, s_hi, s_lo, n, samples)
        cols, send = S.partition_rows(ctx, sh_in, bins, z, *self.splitters, ids=id_col,
                                      id_base=int(ids) if compact else 0, rows=compact)
        ev[1].record()
        del id_col
        cols, recv = S.exchange_partitioned(pg, cols, send)
        ev[2].record()
        src = cols.pop()
        sh, b, zz = (cols if sharded else [None] + cols)
        del cols
        self.table = Z3Table(b, zz, sh, period)
        ev[3].record()
        del sh, b, zz
        if sharded:
            self.table.shards = int(shards) if shards else (
                int(S.all_reduce_scalar(pg, float(self.table.shards or 0), "max")))
        if compact:   # received row r of source rank k: id = base_k + its 4-B row
            bases = torch.tensor([int(ids)], dtype=torch.int64, device=S._device_of(pg))
            allb = [torch.zeros_like(bases) for _ in range(pg.get_world_size())]
            pg.all_gather(allb, bases)
            self._src_rows = src
            self._src_base = torch.cat([v.to(dev) for v in allb])
            self._recv_end = torch.as_tensor(np.cumsum(recv), dtype=torch.int64, device=dev)
            self.src_ids = None
        else:
            self.src_ids = src   # global row id of each received row (the table's perm maps table rows to them)
        self.n = self.table.n
        ev[3].synchronize()
        self.timing = {"partition_ms": ev[0].elapsed_time(ev[1]), "exchange_ms": ev[1].elapsed_time(ev[2]),
                       "sort_ms": ev[2].elapsed_time(ev[3]), "sent_rows": [int(v) for v in send],
                       "received_rows": [int(v) for v in recv]}
        self._bounds()

    def source_ids(self, rows):
        """Global ids of received (slice input) rows."""
        import torch
        if self.src_ids is not None:
            return self.src_ids[rows]
        if self._recv_end is None:   # one slice with contiguous ids
            return rows + self._id_base
        k = torch.searchsorted(self._recv_end, rows, right=True)
        return self._src_base[k] + (self._src_rows[rows].to(torch.int64) & 0xFFFFFFFF)

    def _bounds(self):
        """The slice's first and last key (the clipping bounds)."""
        import torch
        from . import shard as S
        if self.n:
            t = self.table
            ends = torch.tensor([0, self.n - 1], device=t.z.device)
            k_hi, k_lo = S.table_key(None if t.shard is None else t.shard[ends], t.bin[ends], t.z[ends])
            k_hi, k_lo = k_hi.cpu().tolist(), k_lo.cpu().tolist()
            self.kmin, self.kmax = (k_hi[0], k_lo[0]), (k_hi[1], k_lo[1])
        else:
            self.kmin = self.kmax = None

    @classmethod
    def from_points(cls, pg, x, y, t_ms, ids, shard=None, shards=None, period="week", lenient=False, samples=1024):
        bins, z = Z3IndexKeySpace(period).sfc.index_keys(x, y, t_ms, lenient=lenient)
        return cls(pg, bins, z, ids, shard, shards, period, samples)

    def clip(self, arr):
        """gm_key_range rows clipped to this rank's slice."""
        from .shard import clip_key_ranges
        return clip_key_ranges(arr, self.kmin, self.kmax)

    def scan(self, scan_ranges, z3filter=None):
        """(global row ids of this slice's matches, n_match, n_scanned, n_ranges scanned)."""
        arr, _ = key_ranges(scan_ranges, self.table.shards)
        arr = self.clip(arr)
        rows, nm, ns = self.table.scan_key_ranges(arr, z3filter, map_rows=True)   # input rows of the slice
        return self.source_ids(rows), nm, ns, len(arr)

    def query(self, bboxes=None, intervals=None, target=2000):
        """bbox + during query (Z3Filter on the rows of the clipped ranges) on this rank's slice."""
        ks = self.table.ks
        v = ks.get_index_values(bboxes, intervals)
        if v.disjoint:
            import torch
            return torch.zeros(0, dtype=torch.int64, device=self.table.z.device), 0, 0, 0
        return self.scan(ks.get_ranges(v, target=target), F.Z3Filter.from_values(v))


# ---------------------------------------------------------------- Z2 / XZ2 / XZ3 tables
class _KeyTable:
    """Sorted (shard?, bin?, z) key columns of one GPU's slice of an index table (gm_sort_keys), the
    sort's permutation, and the seek + filter of gm_table_scan.  bin None: a key space without a time
    bin ([shard][z BE64]: Z2, XZ2)."""

    def __init__(self, bins, z, shard=None, shards=None):
        import torch
        from .curve import _dev_col
        self.ctx = _lib.context()
        z = _dev_col(z, torch.int64)
        self.n = z.numel()
        dev = z.device
        self.z = torch.empty_like(z)
        self.perm = torch.empty(self.n, dtype=torch.int64, device=dev)
        b_in = None if bins is None else _dev_col(bins, torch.int16)
        self.bin = None if b_in is None else torch.empty_like(b_in)
        self.shard, self.shards, sh_in = None, None, None
        if shard is not None:
            sh_in = torch.as_tensor(np.asarray(shard, np.uint8) if not isinstance(shard, torch.Tensor) else shard,
                                    dtype=torch.uint8).to(dev).contiguous()
            self.shard = torch.empty_like(sh_in)
            self.shards = int(shards) if shards else (int(sh_in.max().item()) + 1 if self.n else 1)
        check(self.ctx.lib.gm_sort_keys(self.ctx.handle, ptr(sh_in), ptr(b_in), ptr(z), self.n, ptr(self.shard),
                                        ptr(self.bin), ptr(self.z), ptr(self.perm)), "gm_sort_keys")

    def key_bytes(self):
        """Row-key prefixes in table order: [shard?][bin BE16][z BE64] or, without a bin, [shard?][z BE64]."""
        import torch
        klen = (1 if self.shard is not None else 0) + (2 if self.bin is not None else 0) + 8
        out = torch.empty((self.n, klen), dtype=torch.uint8, device=self.z.device)
        if self.bin is not None:
            check(self.ctx.lib.gm_z3_key_bytes(self.ctx.handle, ptr(self.shard), ptr(self.bin), ptr(self.z), self.n,
                                               ptr(out)), "gm_z3_key_bytes")
        else:
            check(self.ctx.lib.gm_z2_key_bytes(self.ctx.handle, ptr(self.shard), ptr(self.z), self.n, ptr(out)),
                  "gm_z2_key_bytes")
        return out

    def table_scan(self, arr, flt=None, map_rows=True, ids_cap=None):
        """gm_table_scan over gm_key_range rows `arr` with a ScanFilter (None = no filter): (ids, n_match,
        n_scanned); ids are input rows (map_rows) or table rows."""
        import torch
        arr = np.ascontiguousarray(arr, _lib.KEY_RANGE_DTYPE)
        cap = self.n if ids_cap is None else ids_cap
        ids = torch.empty(max(cap, 1), dtype=torch.int64, device=self.z.device)
        nm, ns = ctypes.c_int64(), ctypes.c_int64()
        rc = self.ctx.lib.gm_table_scan(self.ctx.handle, ptr(self.shard), ptr(self.bin), ptr(self.z), self.n,
                                        arr.ctypes.data if len(arr) else None, len(arr),
                                        ctypes.byref(flt) if flt is not None else None,
                                        ptr(self.perm) if map_rows else None, ptr(ids), cap, ctypes.byref(nm),
                                        ctypes.byref(ns))
        if rc != _lib.GM_E_CAPACITY:
            check(rc, "gm_table_scan")
        return ids[:min(nm.value, cap)], nm.value, ns.value


def _full_filter(cols, boxes, interval=None, t=None):
    """ScanFilter for the XZ full filter: envelope columns x boxes, dtg during (lo, hi) exclusive.  The
    host arrays it points to are returned beside it (they must outlive the call)."""
    f = _lib.ScanFilter()
    keep = []
    if boxes:
        bx = np.ascontiguousarray(np.asarray(boxes, np.float64).reshape(-1, 4))
        keep.append(bx)
        f.xmin, f.ymin, f.xmax, f.ymax = (c.data_ptr() for c in cols)
        f.boxes, f.n_boxes = bx.ctypes.data, len(bx)
    if interval is not None:
        f.during, f.t_ms, f.t_lo, f.t_hi = 1, t.data_ptr(), int(interval[0]), int(interval[1])
    return f, keep


class Z2Table(_KeyTable):
    """A Z2 point index table (Z2IndexKeySpace.scala:48-76: [shard][z BE64]).  query(): ranges
    (getRanges :99-108) -> seek -> Z2Filter on the row keys (the loose bbox, the default), or with
    strict=True the full filter (point in bbox, inclusive, on the x / y columns: useFullFilter :124-130)."""

    def __init__(self, x, y, shard=None, shards=None, lenient=False):
        import torch
        from .curve import _dev_col
        from .keyspace import Z2IndexKeySpace
        self.ks = Z2IndexKeySpace()
        self.x, self.y = _dev_col(x, torch.float64), _dev_col(y, torch.float64)
        super().__init__(None, self.ks.sfc.index(self.x, self.y, lenient=lenient), shard, shards)

    def query(self, bboxes=None, strict=False, target=2000):
        v = self.ks.get_index_values(bboxes)
        if v.disjoint:
            import torch
            return torch.zeros(0, dtype=torch.int64, device=self.z.device), 0, 0
        arr, _ = key_ranges(self.ks.get_ranges(v, target=target), self.shards)
        if strict:
            f, keep = _full_filter((self.x, self.y, self.x, self.y), v.spatialBounds)
        else:
            fb = F.serialize_to_bytes(F.Z2Filter.from_values(v))
            keep = [ctypes.create_string_buffer(fb, len(fb))]
            f = _lib.ScanFilter()
            f.z2filter, f.z2filter_len = ctypes.addressof(keep[0]), len(fb)
        return self.table_scan(arr, f)


class XZ2Table(_KeyTable):
    """An XZ2 index table of geometry envelopes (XZ2IndexKeySpace.scala:48-76: [shard][XZ2 BE64]).
    query(): ranges (getRanges :97-102) -> seek -> the full filter every XZ query applies (:122-125):
    the feature envelope intersects a query box."""

    def __init__(self, xmin, ymin, xmax, ymax, shard=None, shards=None, g=12, lenient=False):
        import torch
        from .curve import _dev_col
        from .keyspace import XZ2IndexKeySpace
        self.ks = XZ2IndexKeySpace(g)
        self.env = tuple(_dev_col(c, torch.float64) for c in (xmin, ymin, xmax, ymax))
        super().__init__(None, self.ks.sfc.index(*self.env, lenient=lenient), shard, shards)

    def query(self, bboxes=None, target=2000, full_filter=True):
        v = self.ks.get_index_values(bboxes)
        if v.disjoint:
            import torch
            return torch.zeros(0, dtype=torch.int64, device=self.z.device), 0, 0
        arr, _ = key_ranges(self.ks.get_ranges(v, target=target), self.shards)
        f, keep = _full_filter(self.env, v.spatialBounds) if full_filter else (None, [])
        return self.table_scan(arr, f)


class XZ3Table(_KeyTable):
    """An XZ3 index table (XZ3IndexKeySpace.scala:60-95: [shard][bin BE16][XZ3 BE64], keys from
    gm_xz3_index_key).  query(): getIndexValues / getRanges (:98-201) -> seek -> the full filter
    (:247-250): envelope intersects a query box AND dtg DURING the interval (exclusive)."""

    def __init__(self, xmin, ymin, xmax, ymax, t_ms, shard=None, shards=None, g=12, period="week", lenient=False):
        import torch
        from .curve import _dev_col, _raise_first, _summary
        from .keyspace import XZ3IndexKeySpace
        self.ks = XZ3IndexKeySpace(period, g)
        self.env = tuple(_dev_col(c, torch.float64) for c in (xmin, ymin, xmax, ymax))
        self.t = _dev_col(t_ms, torch.int64)
        n = self.t.numel()
        ctx = _lib.context()
        b = torch.empty(n, dtype=torch.int16, device=self.t.device)
        xz = torch.empty(n, dtype=torch.int64, device=self.t.device)
        st = _summary()
        check(ctx.lib.gm_xz3_index_key(ctx.handle, *[ptr(c) for c in self.env], ptr(self.t), n, self.ks.sfc.g,
                                       self.ks.period, int(bool(lenient)), ptr(b), ptr(xz), None, ctypes.byref(st)),
              "gm_xz3_index_key")
        _raise_first(st, "XZ3IndexKeySpace.toIndexKey")
        super().__init__(b, xz, shard, shards)

    def query(self, bboxes=None, interval=None, target=2000, full_filter=True):
        """interval: (lo, hi) epoch millis of `dtg DURING lo/hi`, or None."""
        from .keyspace import during
        v = self.ks.get_index_values(bboxes, [during(*interval)] if interval is not None else None)
        if v.disjoint:
            import torch
            return torch.zeros(0, dtype=torch.int64, device=self.z.device), 0, 0
        arr, _ = key_ranges(self.ks.get_ranges(v, target=target), self.shards)
        f, keep = _full_filter(self.env, v.spatialBounds, interval, self.t) if full_filter else (None, [])
        return self.table_scan(arr, f)
