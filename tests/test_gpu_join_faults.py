"""Regression tests for the two round-2 join faults (DESIGN.md §5 "Join faults, round 2").

Both faults were `hipStreamSynchronize: an illegal memory access` in a k_pip_join work-in-progress
tree that had just split the per-wave LDS blob queue into two ends (compact / generic blobs at
01:19, line entries / blobs at 04:10).  The mechanism such a split can produce is an overrun of the
two-ended queue: items of one wave written past its end corrupt the blob references another
wave's slots hold, and item_locate then follows a garbage reference out of the index.  These tests
cover both halves:
  * the queue at capacity with each kind alone and both kinds interleaved, and the Arrow source with
    null slots at tile ends (the second fault's test), all compared with the oracle;
  * a corrupted reference (an imported index whose cell word points far outside the blob array):
    the join's device-side reference check reports GM_E_INDEX instead of faulting the GPU.
"""
import numpy as np
import pytest

from test_gpu_scan_join_ranges import _sorted_pairs, as_np

pytestmark = pytest.mark.gpu

JTILE = 512   # k_pip_join: 256 threads x JILP = 2 points per tile


def _edge_points(ps, offset, rng, n=None):
    """Points a hair inside / outside every polygon edge (line-entry and blob items) and on vertices."""
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    mx, my = 0.5 * (vx[1:] + vx[:-1]), 0.5 * (vy[1:] + vy[:-1])
    dx, dy = vx[1:] - vx[:-1], vy[1:] - vy[:-1]
    ln = np.hypot(dx, dy) + 1e-300
    s = rng.choice([-1.0, 1.0], len(mx))
    px = np.concatenate([mx + s * offset * (-dy / ln), vx])
    py = np.concatenate([my + s * offset * (dx / ln), vy])
    if n is not None:
        k = rng.choice(len(px), n, replace=len(px) < n)
        px, py = px[k], py[k]
    return px, py


def _check(ix, oracle, ps, px, py, modes=("auto",)):
    op = oracle.OraclePolySet(*ps.to_arrays())
    opt, opl = op.join(px, py, nthreads=8)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    for mode in modes:
        pt, pl = ix.join(px, py, mode=mode)   # raises GeomesaHipError on GM_E_INDEX
        assert np.array_equal(_sorted_pairs(pt, pl), exp), mode


def test_queue_full_of_line_items(gpu, oracle):
    """Every point of every wave in a crossed cell, a hair off its segment: each item step queues 64
    line-entry items, so every step runs an evaluation round at the queue's 64-item threshold."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(20, 10)
    px, py = _edge_points(ps, 1e-4, np.random.default_rng(3), 64 * JTILE + 5)
    _check(PolygonIndex(ps), oracle, ps, px, py)


def test_queue_full_of_blob_items(gpu, oracle):
    """A coarse grid (1 cell per polygon): every cell holds many segments, so every item is a generic
    blob (and some rings fall back to the slab walk) -- the queue's other end at capacity."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(20, 10)
    px, py = synthetic_points(40 * JTILE + 3, seed=7)
    ix = PolygonIndex(ps, cells_per_poly=1)
    assert ix.stats()["slow"] > 0
    _check(ix, oracle, ps, px, py)


@pytest.mark.parametrize("block", [1, 31, 32, 33, 64])
def test_queue_both_kinds_interleaved(gpu, oracle, block):
    """Line-entry items (edge points) and blob items (vertices: on the boundary, so the line entry
    defers to the blob) interleaved in runs of `block` points, so both ends of each wave's queue fill
    together up to the 128-slot capacity, in every proportion."""
    from geomesa_amd.join import PolygonIndex, synthetic_counties
    ps = synthetic_counties(20, 10)
    rng = np.random.default_rng(block)
    ppo, pro, rvo, vx, vy = ps.to_arrays()
    ex, ey = _edge_points(ps, 1e-4, rng, 48 * JTILE)
    k = rng.choice(len(vx), 48 * JTILE)
    bx, by = vx[k], vy[k]
    px = np.empty(48 * JTILE); py = np.empty(48 * JTILE)
    idx = np.arange(48 * JTILE)
    take_edge = (idx // block) % 2 == 0
    px[take_edge], py[take_edge] = ex[:take_edge.sum()], ey[:take_edge.sum()]
    px[~take_edge], py[~take_edge] = bx[:(~take_edge).sum()], by[:(~take_edge).sum()]
    _check(PolygonIndex(ps), oracle, ps, px, py)


@pytest.mark.parametrize("f32", [False, True])
def test_arrow_nulls_at_tile_ends(gpu, oracle, f32):
    """The second fault's case (Arrow point column, direct join): null slots at every tile boundary and
    the first / last row, a row count that leaves a partial last tile, boundary-heavy points."""
    from geomesa_amd import arrow
    from geomesa_amd.join import synthetic_counties, synthetic_points
    from test_gpu_arrow import point_array, polyset_to_arrow
    ps = synthetic_counties(12, 6)
    rng = np.random.default_rng(5)
    ex, ey = _edge_points(ps, 1e-4, rng, 20 * JTILE)
    rx, ry = synthetic_points(20 * JTILE + 77, seed=9)
    px, py = np.concatenate([ex, rx]), np.concatenate([ey, ry])
    if f32:   # a Float4 column widens its floats: the oracle sees the same widened values
        px, py = px.astype(np.float32).astype(np.float64), py.astype(np.float32).astype(np.float64)
    n = len(px)
    nulls = rng.uniform(size=n) < 0.05
    for t in range(0, n, JTILE):
        nulls[t] = True
        nulls[min(n - 1, t + JTILE - 1)] = True
    nulls[-1] = True
    idx = arrow.ArrowPolygonIndex(polyset_to_arrow(ps), kind="multipolygon")   # polygons stay Float8
    pt, pl = idx.join(point_array(px, py, nulls, f32=f32), mode="auto")
    got = set(zip(as_np(pt).tolist(), as_np(pl).tolist()))
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=8)
    exp = {(a, b) for a, b in zip(opt.tolist(), opl.tolist()) if not nulls[a]}
    assert got == exp


def test_corrupt_reference_reports_instead_of_faulting(gpu):
    """What the faulting trees did -- follow a blob reference that points outside the index -- now
    ends in GM_E_INDEX (device-side reference check) in the join, the row predicate and the fused
    query scan, and the context and a healthy index keep working afterwards."""
    import torch
    from geomesa_amd import _lib
    from geomesa_amd.join import PolygonIndex, synthetic_counties, synthetic_points
    ps = synthetic_counties(20, 10)
    good = PolygonIndex(ps)
    lay, arrs = good.export_arrays()
    gx, gy = int(lay.dims[0]), int(lay.dims[1])
    x0, y0, _, _, icw, ich = (float(v) for v in lay.grid)
    px, py = synthetic_points(50_000, seed=11)
    cx = np.clip(((px[:64] - x0) * icw).astype(np.int64), 0, gx - 1)
    cy = np.clip(((py[:64] - y0) * ich).astype(np.int64), 0, gy - 1)
    cw = arrs[3].view(torch.int32)   # cell words (gm_pip_index_layout order: rings, slab_off, slab_edges, cell_word, ...)
    bad_word = (1 << 30) | 0x1FFFFFF0   # BOUNDARY, generic blob at 16-B offset 0x1FFFFFF0: far outside the blob array
    assert int(lay.bytes[7]) // 16 < 0x1FFFFFF0
    cells = torch.as_tensor(cy * gx + cx, device=cw.device)
    cw[cells] = torch.tensor(bad_word - (1 << 32) if bad_word >= 1 << 31 else bad_word, dtype=torch.int32,
                             device=cw.device)
    bad = PolygonIndex.from_arrays(lay, arrs, polyset=ps)
    from geomesa_amd.filters import query_scan
    calls = {"join": lambda: bad.join(px, py),
             "join count": lambda: bad.join(px, py, count_only=True),
             "relate": lambda: bad.relate(np.zeros(len(px), np.int32), px, py),
             "query": lambda: query_scan(px, py, geoms=bad, op="intersects")}
    for name, call in calls.items():
        with pytest.raises(_lib.GeomesaHipError) as ei:
            call()
        assert "reference check" in str(ei.value), name
    # a stream-ordered join (no pair count asked) reports at the next synchronising call, once
    import ctypes
    x = torch.as_tensor(px, device="cuda"); y = torch.as_tensor(py, device="cuda")
    pt0 = torch.empty(len(px) * 2, dtype=torch.int64, device="cuda")
    pl0 = torch.empty(len(px) * 2, dtype=torch.int32, device="cuda")
    rc = bad.ctx.lib.gm_pip_join_ex(bad.ctx.handle, bad._h, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                                    len(px), 0, ctypes.c_void_p(pt0.data_ptr()), ctypes.c_void_p(pl0.data_ptr()),
                                    len(px) * 2, None, _lib.GM_JOIN_AUTO)
    assert rc == _lib.GM_OK
    with pytest.raises(_lib.GeomesaHipError) as ei:
        bad.ctx.sync()
    assert "reference check" in str(ei.value)
    assert "gm_pip_join" in str(ei.value) and "gm_pip_relate" not in str(ei.value)   # names the call that raised it
    bad.ctx.sync()   # cleared once reported
    # a stream-ordered row predicate on the bad index, read by a later synchronising join on the
    # healthy one: the text names the row predicate as a possible source
    rid = torch.zeros(len(px), dtype=torch.int32, device="cuda")
    loc = torch.empty(len(px), dtype=torch.uint8, device="cuda")
    assert bad.ctx.lib.gm_pip_relate(bad.ctx.handle, bad._h, ctypes.c_void_p(rid.data_ptr()), ctypes.c_void_p(x.data_ptr()),
                                     ctypes.c_void_p(y.data_ptr()), len(px), ctypes.c_void_p(loc.data_ptr())) == _lib.GM_OK
    with pytest.raises(_lib.GeomesaHipError) as ei:
        bad.ctx.sync()
    assert "gm_pip_relate" in str(ei.value)
    # the healthy index on the same context is unaffected
    pt, pl = good.join(px, py)
    pt2, pl2 = PolygonIndex.from_arrays(*good.export_arrays(), polyset=ps).join(px, py)
    assert np.array_equal(_sorted_pairs(pt, pl), _sorted_pairs(pt2, pl2))
