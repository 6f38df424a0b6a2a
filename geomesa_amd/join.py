"""st_contains point-in-polygon join on the GPU (JTS 1.20 Geometry.contains semantics).

Replaces the per-pair UDF evaluation of the Spark-SQL spatial join:
  SQLRules.SpatialJoinStrategy -> GeoMesaJoinRelation.sweeplineJoin -> OverlapAction.overlap ->
  ST_Contains(geom1, geom2) = geom1.contains(geom2)
(geomesa-spark/geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91, OverlapAction.scala:25-41,
 geomesa-spark/geomesa-spark-jts/.../udf/SpatialRelationFunctions.scala:29,94).

Polygons travel as CSR (polygon -> parts -> rings -> vertices, rings closed).  Points are device
columns.  The result is the set of (point id, polygon id) pairs; like the reference RDD it is
unordered (tests compare as sets).  `st_contains(poly, point)` of a null argument is null
(SQLFunctionHelper.nullableUDF, SQLFunctionHelper.scala:27-33) -- here: rows flagged null are
skipped by the caller.
"""
import ctypes
import re

import numpy as np

from . import _lib
from ._lib import check, ptr


class PolygonSet:
    """CSR polygon set.  `polys` is a list of polygons; a polygon is a list of parts; a part is a
    list of rings (shell first); a ring is an (k, 2) array-like of vertices (closed or not -- it is
    closed here the way JTS LinearRing requires)."""

    def __init__(self, poly_part_off, part_ring_off, ring_vert_off, vx, vy):
        self.poly_part_off = np.ascontiguousarray(poly_part_off, np.int32)
        self.part_ring_off = np.ascontiguousarray(part_ring_off, np.int32)
        self.ring_vert_off = np.ascontiguousarray(ring_vert_off, np.int32)
        self.vx = np.ascontiguousarray(vx, np.float64)
        self.vy = np.ascontiguousarray(vy, np.float64)

    @property
    def n_polys(self):
        return len(self.poly_part_off) - 1

    @property
    def n_vertices(self):
        return len(self.vx)

    @classmethod
    def from_polygons(cls, polys):
        ppo, pro, rvo, vx, vy = [0], [0], [0], [], []
        for poly in polys:
            for part in poly:
                for ring in part:
                    r = np.asarray(ring, np.float64).reshape(-1, 2)
                    if len(r) and (r[0, 0] != r[-1, 0] or r[0, 1] != r[-1, 1]):
                        r = np.vstack([r, r[:1]])
                    vx.append(r[:, 0]); vy.append(r[:, 1])
                    rvo.append(rvo[-1] + len(r))
                pro.append(len(rvo) - 1)
            ppo.append(len(pro) - 1)
        vx = np.concatenate(vx) if vx else np.zeros(0)
        vy = np.concatenate(vy) if vy else np.zeros(0)
        return cls(ppo, pro, rvo, vx, vy)

    @classmethod
    def from_wkt(cls, wkts):
        return cls.from_polygons([parse_wkt_polygon(w) for w in wkts])

    def c_struct(self):
        return _lib.PolySetC(self.n_polys, self.poly_part_off.ctypes.data, self.part_ring_off.ctypes.data,
                             self.ring_vert_off.ctypes.data, self.vx.ctypes.data, self.vy.ctypes.data)

    def to_arrays(self):
        return (self.poly_part_off, self.part_ring_off, self.ring_vert_off, self.vx, self.vy)


_num = r"[-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?"


def _ring(s):
    pts = [tuple(float(v) for v in p.split()) for p in s.split(",")]
    return np.array([(p[0], p[1]) for p in pts], np.float64)


def parse_wkt_polygon(wkt):
    """POLYGON / MULTIPOLYGON WKT -> list of parts -> list of rings."""
    w = wkt.strip()
    up = w.upper()
    if up.startswith("MULTIPOLYGON"):
        body = w[w.index("(") + 1:w.rindex(")")]
        parts = re.findall(r"\(\s*(\(.*?\)(?:\s*,\s*\(.*?\))*)\s*\)", body)
        return [[_ring(r) for r in re.findall(r"\(([^()]*)\)", p)] for p in parts]
    if up.startswith("POLYGON"):
        body = w[w.index("(") + 1:w.rindex(")")]
        return [[_ring(r) for r in re.findall(r"\(([^()]*)\)", body)]]
    raise ValueError("not a polygon: %s" % wkt[:40])


class PolygonIndex:
    """Device-side join index for a PolygonSet (gm_pip_index_create)."""

    def __init__(self, polyset, ctx=None, cells_per_poly=0):
        self.polyset = polyset
        self.ctx = ctx or _lib.context()
        self._cs = polyset.c_struct()
        self._h = ctypes.c_void_p()
        check(self.ctx.lib.gm_pip_index_create_ex(self.ctx.handle, ctypes.byref(self._cs), int(cells_per_poly),
                                                  ctypes.byref(self._h)), "gm_pip_index_create_ex")

    def export_arrays(self):
        """(layout, [uint8 device tensors]) of this index: what another GPU needs to rebuild it with
        `from_arrays` (gm_pip_index_export / gm_pip_index_copy_array)."""
        import torch
        lay = _lib.PipIndexLayout()
        check(self.ctx.lib.gm_pip_index_export(self._h, ctypes.byref(lay)), "gm_pip_index_export")
        dev = torch.device("cuda", self.ctx.device)
        arrs = []
        for k in range(_lib.GM_PIP_INDEX_ARRAYS):
            t = torch.empty(max(int(lay.bytes[k]), 1), dtype=torch.uint8, device=dev)
            check(self.ctx.lib.gm_pip_index_copy_array(self.ctx.handle, self._h, k, ptr(t)), "gm_pip_index_copy_array")
            arrs.append(t)
        return lay, arrs

    @classmethod
    def from_arrays(cls, layout, arrays, ctx=None, polyset=None):
        """An index rebuilt from another GPU's export (device tensors on this rank's GPU)."""
        self = cls.__new__(cls)
        self.polyset = polyset
        self.ctx = ctx or _lib.context()
        self._cs = None
        self._h = ctypes.c_void_p()
        ptrs = (ctypes.c_void_p * _lib.GM_PIP_INDEX_ARRAYS)(*[a.data_ptr() for a in arrays])
        check(self.ctx.lib.gm_pip_index_import(self.ctx.handle, ctypes.byref(layout), ptrs, ctypes.byref(self._h)),
              "gm_pip_index_import")
        return self

    def stats(self):
        """Index statistics: cells, (cell, polygon) entries, boundary entries, ring records,
        slow-walk records, blob bytes, compact blobs."""
        import numpy as np
        st = np.zeros(7, np.int64)
        check(self.ctx.lib.gm_pip_index_stats(self._h, st.ctypes.data), "gm_pip_index_stats")
        return dict(zip(["cells", "entries", "boundary", "records", "slow", "blob_bytes", "compact"], st.tolist()))

    CENSUS = ["points", "outside", "coarse_empty", "coarse_interior", "coarse_raw_mixed", "fine", "fine_empty",
              "fine_interior", "fine_line", "fine_compact", "fine_generic", "fine_list", "list_entries",
              "list_blobs", "line_resolved", "line_fallback", "fine_inline", "inline_fallback", "coarse_gather",
              "fine_inline2"]

    def census(self, px, py):
        """Diagnostic: how the lookup chain resolves these points, stage by stage (gm_pip_join_census)."""
        import numpy as np
        import torch
        dev = torch.device("cuda", self.ctx.device)
        x = torch.as_tensor(px, dtype=torch.float64, device=dev).contiguous()
        y = torch.as_tensor(py, dtype=torch.float64, device=dev).contiguous()
        c = np.zeros(len(self.CENSUS), np.int64)
        check(self.ctx.lib.gm_pip_join_census(self.ctx.handle, self._h, ptr(x), ptr(y), x.numel(), c.ctypes.data),
              "gm_pip_join_census")
        return dict(zip(self.CENSUS, c.tolist()))

    MODES = {"auto": _lib.GM_JOIN_AUTO, "direct": _lib.GM_JOIN_DIRECT}

    PREDICATES = {"st_contains": _lib.GM_SPATIAL_CONTAINS, "st_within": _lib.GM_SPATIAL_CONTAINS,
                  "st_intersects": _lib.GM_SPATIAL_INTERSECTS, "st_covers": _lib.GM_SPATIAL_INTERSECTS}

    def join(self, px, py, id_base=0, cap=None, count_only=False, mode="auto", predicate="st_contains"):
        """Returns (pt_ids, poly_ids) device tensors (or the pair count when count_only).

        mode: "auto" or "direct" (the staged direct pass over the point columns; the two are one
        strategy on MI355X).  predicate: the join condition's UDF,
        st_contains(polygon, point) / st_within(point, polygon) or st_intersects / st_covers."""
        m = self.MODES[mode]
        pr = self.PREDICATES[predicate]
        import torch
        from .curve import _dev_col
        px = _dev_col(px, torch.float64)
        py = _dev_col(py, torch.float64)
        n = px.numel()
        npairs = ctypes.c_int64()
        if count_only:
            check(self.ctx.lib.gm_pip_join_pred(self.ctx.handle, self._h, ptr(px), ptr(py), n, id_base, None, None,
                                                0, ctypes.byref(npairs), m, pr), "gm_pip_join")
            return npairs.value
        if cap is None:
            cap = max(1024, n + n // 4)
        while True:
            pt = torch.empty(cap, dtype=torch.int64, device=px.device)
            pl = torch.empty(cap, dtype=torch.int32, device=px.device)
            rc = self.ctx.lib.gm_pip_join_pred(self.ctx.handle, self._h, ptr(px), ptr(py), n, id_base, ptr(pt),
                                               ptr(pl), cap, ctypes.byref(npairs), m, pr)
            if rc == _lib.GM_E_CAPACITY:
                cap = npairs.value
                continue
            check(rc, "gm_pip_join")
            k = npairs.value
            return pt[:k], pl[:k]

    def relate(self, poly_ids, px, py):
        """Per-row location of point i in polygon poly_ids[i] (LOC_EXTERIOR / BOUNDARY / INTERIOR, or
        LOC_NULL where poly_ids[i] < 0 marks a null row): the row-wise UDF path (gm_pip_relate)."""
        import torch
        from .curve import _dev_col
        px = _dev_col(px, torch.float64)
        py = _dev_col(py, torch.float64)
        pid = _dev_col(poly_ids, torch.int64).to(torch.int32)
        n = px.numel()
        if py.numel() != n or pid.numel() != n:
            raise ValueError("poly_ids, px and py must have one entry per row")
        loc = torch.empty(n, dtype=torch.uint8, device=px.device)
        check(self.ctx.lib.gm_pip_relate(self.ctx.handle, self._h, ptr(pid), ptr(px), ptr(py), n, ptr(loc)),
              "gm_pip_relate")
        self.ctx.sync()   # the call is stream-ordered: a failed device reference check surfaces here
        return loc

    def predicate(self, name, poly_ids, px, py):
        """Spark SQL's st_* relation UDF row by row (SpatialRelationFunctions.scala:29-37) for
        (polygon, point) rows: returns (value, is_null) bool device tensors (nullableUDF: a null
        argument gives null, SQLFunctionHelper.scala:27-33).  st_within takes (point, polygon)."""
        loc = self.relate(poly_ids, px, py)
        return ROW_PREDICATES[name](loc), loc == LOC_NULL

    def close(self):
        if self._h:
            self.ctx.lib.gm_pip_index_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


LOC_EXTERIOR, LOC_BOUNDARY, LOC_INTERIOR, LOC_NULL = 0, 1, 2, 255

# DE-9IM predicates of (areal geometry, point) as functions of PointLocator's location
ROW_PREDICATES = {
    "st_contains": lambda l: l == LOC_INTERIOR,
    "st_within": lambda l: l == LOC_INTERIOR,        # st_within(point, polygon)
    "st_covers": lambda l: (l == LOC_INTERIOR) | (l == LOC_BOUNDARY),
    "st_intersects": lambda l: (l == LOC_INTERIOR) | (l == LOC_BOUNDARY),
    "st_touches": lambda l: l == LOC_BOUNDARY,
    "st_disjoint": lambda l: l == LOC_EXTERIOR,
    "st_crosses": lambda l: l != l,                  # a point cannot cross an area (IM T*****T** needs 2 points)
    "st_overlaps": lambda l: l != l,                 # different dimensions
    "st_equals": lambda l: l != l,
}


def st_contains_join(polyset, px, py):
    """All (point, polygon) pairs with st_contains(polygon, point) = true."""
    return PolygonIndex(polyset).join(px, py)


# ------------------------------------------------------------------------------ synthetic inputs

CONUS = (-125.0, 24.0, -66.0, 50.0)


def synthetic_counties(nx=80, ny=40, seed=0x67656f6d65736121, box=CONUS, vmin=64, vmax=256,
                       hole_frac=0.10, multi_frac=0.05):
    """Seeded jittered nx x ny grid of star-shaped 'county' polygons (BASELINE config 4).

    Each polygon lies inside its own grid cell, so neighbours share no edges and contains() is
    order independent; ~hole_frac get a hole, ~multi_frac are 2-part MultiPolygons."""
    rng = np.random.default_rng(seed & 0xFFFFFFFFFFFFFFFF)
    x0, y0, x1, y1 = box
    cw, ch = (x1 - x0) / nx, (y1 - y0) / ny
    R = 0.45 * min(cw, ch)
    polys = []
    for j in range(ny):
        for i in range(nx):
            cx = x0 + (i + 0.5) * cw + rng.uniform(-0.03, 0.03) * R
            cy = y0 + (j + 0.5) * ch + rng.uniform(-0.03, 0.03) * R
            nv = int(rng.integers(vmin, vmax + 1))
            ang = np.sort(rng.uniform(0, 2 * np.pi, nv))
            rad = R * (0.6 + 0.35 * rng.uniform(0, 1, nv))
            shell = np.stack([cx + rad * np.cos(ang), cy + rad * np.sin(ang)], 1)
            rings = [shell]
            if rng.uniform() < hole_frac:
                hn = int(rng.integers(8, 32))
                ha = np.sort(rng.uniform(0, 2 * np.pi, hn))
                hr = 0.25 * R * (0.5 + 0.5 * rng.uniform(0, 1, hn))
                rings.append(np.stack([cx + hr * np.cos(ha), cy + hr * np.sin(ha)], 1))
            parts = [rings]
            if rng.uniform() < multi_frac:
                k = int(rng.integers(0, 4))
                ux, uy = (1 if k & 1 else -1) * cw / 2, (1 if k & 2 else -1) * ch / 2
                nrm = np.hypot(ux, uy)
                d = 0.82 * nrm
                px_, py_ = cx + ux / nrm * d, cy + uy / nrm * d
                sn = int(rng.integers(8, 24))
                sa = np.sort(rng.uniform(0, 2 * np.pi, sn))
                sr = 0.05 * R * (0.6 + 0.4 * rng.uniform(0, 1, sn))
                parts.append([np.stack([px_ + sr * np.cos(sa), py_ + sr * np.sin(sa)], 1)])
            polys.append(parts)
    return PolygonSet.from_polygons(polys)


def synthetic_points(n, seed=0x67656f6d65736121, box=CONUS):
    rng = np.random.default_rng((seed + 1) & 0xFFFFFFFFFFFFFFFF)
    x0, y0, x1, y1 = box
    return rng.uniform(x0, x1, n), rng.uniform(y0, y1, n)
