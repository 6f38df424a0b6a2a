"""The oracle's orientation and point location against exact rational arithmetic (CPU only).

JTS decides orientation with CGAlgorithmsDD.orientationIndex (a 1e-15 filter, then double-double)
and locates a point with RayCrossingCounter (a point on an edge is BOUNDARY; otherwise crossing
parity per ring) combined over a MultiPolygon's parts by the Mod-2 boundary rule (PointLocator).
The oracle restates those operation for operation (gm_oracle.c gmo_orientation_index, gmo_locate).
Here both are checked against Python's `fractions.Fraction` -- the exact sign of the orientation
determinant, the exact on-edge test and exact crossing parity -- on inputs built to sit on or next
to edges: points on segments rounded to the nearest double and nudged by 1-3 ulps, and lattice
polygons whose lattice points fall exactly on their edges.  Where the double-double result is exact
(every case here), JTS, the oracle and exact arithmetic must agree, so these cases pin the
boundary / near-collinear behaviour that the reference's own box KATs leave open.
"""
import functools
from fractions import Fraction as F

import numpy as np
import pytest

from geomesa_amd.join import PolygonSet

LOC_EXTERIOR, LOC_BOUNDARY, LOC_INTERIOR = 0, 1, 2


def _orient_exact(ax, ay, bx, by, qx, qy):
    d = (F(bx) - F(ax)) * (F(qy) - F(ay)) - (F(by) - F(ay)) * (F(qx) - F(ax))
    return (d > 0) - (d < 0)


def test_orientation_index_near_collinear(oracle):
    rng = np.random.default_rng(5)
    n = 40_000
    ax, bx = rng.uniform(-180, 180, n), rng.uniform(-180, 180, n)
    ay, by = rng.uniform(-90, 90, n), rng.uniform(-90, 90, n)
    t = rng.uniform(0, 1, n)
    qx, qy = ax + t * (bx - ax), ay + t * (by - ay)       # on the segment, rounded to a double
    k = rng.integers(-3, 4, n)
    which = rng.integers(0, 2, n)
    for i in range(n):                                    # nudged by |k| ulps along one axis
        for _ in range(abs(int(k[i]))):
            if which[i]:
                qx[i] = np.nextafter(qx[i], np.inf if k[i] > 0 else -np.inf)
            else:
                qy[i] = np.nextafter(qy[i], np.inf if k[i] > 0 else -np.inf)
    # plus exactly collinear triples (integer and dyadic coordinates)
    m = 5_000
    ix, iy = rng.integers(-1000, 1000, m).astype(np.float64) / 8, rng.integers(-1000, 1000, m).astype(np.float64) / 8
    sx, sy = rng.integers(-50, 50, m).astype(np.float64) / 4, rng.integers(-50, 50, m).astype(np.float64) / 4
    s = rng.integers(-4, 5, m).astype(np.float64)
    cases = [(ax[i], ay[i], bx[i], by[i], qx[i], qy[i]) for i in range(n)]
    cases += [(ix[i], iy[i], ix[i] + sx[i], iy[i] + sy[i], ix[i] + s[i] * sx[i], iy[i] + s[i] * sy[i]) for i in range(m)]
    zeros = 0
    for c in cases:
        a, b, q = (float(c[0]), float(c[1])), (float(c[2]), float(c[3])), (float(c[4]), float(c[5]))
        e = _orient_exact(*a, *b, *q)
        got = oracle.orientation_index(*a, *b, *q)
        assert got == e, (a, b, q, got, e)
        zeros += e == 0
    assert zeros >= m   # the collinear triples (and some rounded ones) really are collinear


def _locate_ring_exact(ring, x, y):
    """BOUNDARY if (x, y) is on an edge, else crossing parity (1 = inside), exactly."""
    X, Y = F(x), F(y)
    inside = False
    for k in range(len(ring) - 1):
        ax, ay = F(ring[k][0]), F(ring[k][1])
        bx, by = F(ring[k + 1][0]), F(ring[k + 1][1])
        cross = (bx - ax) * (Y - ay) - (by - ay) * (X - ax)
        if cross == 0 and min(ax, bx) <= X <= max(ax, bx) and min(ay, by) <= Y <= max(ay, by):
            return LOC_BOUNDARY
        if (ay > Y) != (by > Y):
            xi = ax + (Y - ay) * (bx - ax) / (by - ay)
            if xi > X:
                inside = not inside
    return LOC_INTERIOR if inside else LOC_EXTERIOR


def _locate_exact(parts, x, y):
    """PointLocator over a (Multi)Polygon: per part, on a ring -> BOUNDARY, in the shell and no hole
    -> INTERIOR; parts combined by the Mod-2 rule (an odd count of boundary parts is BOUNDARY)."""
    is_in, nb = False, 0
    for rings in parts:
        locs = [_locate_ring_exact(r, x, y) for r in rings]
        if LOC_BOUNDARY in locs:
            nb += 1
        elif locs[0] == LOC_INTERIOR and all(l == LOC_EXTERIOR for l in locs[1:]):
            is_in = True
    if nb % 2 == 1:
        return LOC_BOUNDARY
    return LOC_INTERIOR if (nb > 0 or is_in) else LOC_EXTERIOR


def _closed(r):
    r = [tuple(map(float, v)) for v in r]
    return r + [r[0]] if r[0] != r[-1] else r


def lattice_polys():
    """Lattice polygons (vertices on multiples of 1/4, slanted edges of several slopes, holes,
    MultiPolygons whose parts share an edge or touch at a vertex)."""
    return [
        [[_closed([(0, 0), (4, 0), (4, 3), (0, 3)]), _closed([(1, 1), (2, 1), (1.5, 2)])]],          # square + hole
        [[_closed([(0, 0), (3, 1), (5, 4), (1, 3.5)])]],                                            # slanted quad
        [[_closed([(0, 0), (2, 0), (2, 2), (0, 2)])], [_closed([(2, 0), (4, 0), (4, 2), (2, 2)])]],    # shared edge
        [[_closed([(0, 0), (2, 0), (2, 2), (0, 2)])], [_closed([(2, 2), (4, 2), (4, 4), (2, 4)])]],    # shared vertex
        [[_closed([(0, 0), (6, 0), (6, 1), (1, 1), (1, 2), (6, 2), (6, 3), (0, 3)])]],              # concave E
        [[_closed([(0, 0), (5, 0.75), (2.5, 4.25), (0.25, 2.5)]), _closed([(1, 1), (2.5, 1.25), (1.75, 2.5)])]],
    ]


def stacked_polys():
    """24 polygons stacked over one region (nested squares, diamonds with slanted edges, squares with
    a hole, two-part MultiPolygons): cells in the middle list 15 or more polygons, the long-list
    encoding (LIST_LONG, a count slot before the entries)."""
    polys = []
    for k in range(8):
        a = 0.25 * k
        polys.append([[_closed([(a, a), (6 - a, a), (6 - a, 6 - a), (a, 6 - a)])]])                 # nested squares
        c = 3.0
        r = 3.0 - 0.25 * k
        polys.append([[_closed([(c - r, c), (c, c - r), (c + r, c), (c, c + r)])]])                 # diamonds
        h = 0.5 + 0.125 * k
        polys.append([[_closed([(1, 1), (5, 1), (5, 5), (1, 5)]), _closed([(3 - h, 3 - h), (3 + h, 3 - h), (3, 3 + h)])],
                      [_closed([(5.5, 0.25 * k), (6.5, 0.25 * k), (6.5, 0.25 * k + 1), (5.5, 0.25 * k + 1)])]])
    return polys


LATTICE = np.arange(-1, 7.01, 0.125)   # lattice points on multiples of 1/8


@functools.lru_cache(maxsize=None)
def exact_lattice(which):
    """(polygons, x, y, exact location [polygon, point]) of every LATTICE point, computed once per set
    (the GPU tests reuse it across grid densities)."""
    polys = lattice_polys() if which == "lattice" else stacked_polys()
    gx, gy = np.meshgrid(LATTICE, LATTICE)
    x, y = gx.ravel().copy(), gy.ravel().copy()
    loc = np.array([[_locate_exact(parts, float(a), float(b)) for a, b in zip(x, y)] for parts in polys], np.uint8)
    return polys, x, y, loc


@pytest.mark.parametrize("which", ["lattice", "stacked"])
def test_locate_lattice_polygons_exact(oracle, which):
    """lattice_polys() / stacked_polys() against every lattice point: many lie exactly on edges,
    vertices and shared edges."""
    polys = lattice_polys() if which == "lattice" else stacked_polys()
    ps = PolygonSet.from_polygons(polys)
    ops = oracle.OraclePolySet(*ps.to_arrays())
    g = LATTICE
    counts = {LOC_EXTERIOR: 0, LOC_BOUNDARY: 0, LOC_INTERIOR: 0}
    for p, parts in enumerate(polys):
        for x in g:
            for y in g:
                e = _locate_exact(parts, float(x), float(y))
                got = ops.locate(p, float(x), float(y))
                assert got == e, (p, x, y, got, e)
                counts[e] += 1
                # st_contains = interior, st_intersects / st_covers = not exterior
                assert ops.contains(p, float(x), float(y)) == (e == LOC_INTERIOR)
                assert ops.intersects(p, float(x), float(y)) == (e != LOC_EXTERIOR)
    assert counts[LOC_BOUNDARY] > 300 and counts[LOC_INTERIOR] > 1000 and counts[LOC_EXTERIOR] > 1000, counts
