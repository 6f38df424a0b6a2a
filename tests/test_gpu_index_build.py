"""The join index built on the device (GM_PARAM_INDEX_BUILD = 0, the default) against the host build
(= 1): the eight exported arrays must be byte-identical and the statistics equal, over the synthetic
counties (holes, MultiPolygons), the US-state shapefile fixture, polygons with more edges than the
build kernel's LDS band (its global-band path), several grid densities, and a row wider than one
256-cell segment.  The joins themselves are checked against the oracle by the other join tests,
which now run on device-built indexes."""
import numpy as np
import pytest

from shapefile import us_states

pytestmark = pytest.mark.gpu


def _build(ps, cells, host):
    from geomesa_amd import _lib
    from geomesa_amd.join import PolygonIndex
    ctx = _lib.context()
    try:
        ctx.set_param(_lib.GM_PARAM_INDEX_BUILD, 1 if host else 0)
        ix = PolygonIndex(ps, ctx, cells)
    finally:
        ctx.set_param(_lib.GM_PARAM_INDEX_BUILD, 0)
    return ix


def _compare(ps, cells):
    d, h = _build(ps, cells, False), _build(ps, cells, True)
    assert d.stats() == h.stats()
    ld, ad = d.export_arrays()
    lh, ah = h.export_arrays()
    assert bytes(ld) == bytes(lh)
    names = ["rings", "slab_off", "slab_edges", "cell_word", "coarse_word", "compact", "list_ent", "blob"]
    for k, (x, y) in enumerate(zip(ad, ah)):
        assert x.numel() == y.numel(), names[k]
        assert bool((x == y).all()), names[k]
    return d


def _star_polys(nv, n, rng, holes=False):
    polys = []
    for j in range(n):
        cx, cy = -100 + 6 * j, 38.0
        ang = np.sort(rng.uniform(0, 2 * np.pi, nv))
        rad = 2.5 * (0.5 + 0.5 * rng.uniform(0, 1, nv))
        rings = [np.stack([cx + rad * np.cos(ang), cy + rad * np.sin(ang)], 1)]
        if holes:
            ha = np.sort(rng.uniform(0, 2 * np.pi, 40))
            rings.append(np.stack([cx + 0.3 * np.cos(ha), cy + 0.3 * np.sin(ha)], 1))
        polys.append([rings])
    return polys


@pytest.mark.parametrize("grid,cells", [((20, 10), 0), ((20, 10), 512), ((40, 20), 8192), ((80, 40), 0)])
def test_device_build_matches_host_counties(gpu, grid, cells):
    from geomesa_amd.join import synthetic_counties
    _compare(synthetic_counties(*grid), cells)


@pytest.mark.parametrize("cells", [0, 2048])
def test_device_build_matches_host_states(gpu, cells):
    _compare(us_states()[0], cells)


def test_device_build_matches_host_large_rings(gpu):
    """3,000-vertex rings (band beyond the LDS capacity) with holes, and a 4-polygon set whose grid
    rows are several 256-cell segments wide."""
    from geomesa_amd.join import PolygonSet
    rng = np.random.default_rng(4)
    _compare(PolygonSet.from_polygons(_star_polys(3000, 3, rng, holes=True)), 0)
    _compare(PolygonSet.from_polygons(_star_polys(200, 4, rng)), 200_000)


def test_device_build_join_equals_oracle(gpu, oracle):
    from geomesa_amd.join import PolygonSet, synthetic_points
    rng = np.random.default_rng(8)
    ps = PolygonSet.from_polygons(_star_polys(3000, 3, rng, holes=True))
    ix = _compare(ps, 0)
    px, py = synthetic_points(400_000, seed=3, box=(-104, 34, -82, 42))
    from test_gpu_scan_join_ranges import _sorted_pairs
    opt, opl = oracle.OraclePolySet(*ps.to_arrays()).join(px, py, nthreads=16)
    exp = np.stack([opt, opl.astype(np.int64)], 1)
    exp = exp[np.lexsort((exp[:, 1], exp[:, 0]))]
    assert np.array_equal(_sorted_pairs(*ix.join(px, py)), exp)
