"""Minimal ESRI shapefile reader for the test fixtures (tests/golden/us_state): polygon records
(.shp shape types 5 / 15 / 25) as a join.PolygonSet, and the attribute table (.dbf, dBASE III).

The fixture is the reference's own test data (geomesa-convert/geomesa-convert-shp/src/test/resources/
us_state/cb_2017_us_state_20m.shp: 52 records, 132 rings, 13,832 vertices).  Rings follow the
shapefile convention read by GeoTools' PolygonHandler: clockwise rings are shells, counter-clockwise
rings are holes and belong to the first shell whose envelope holds them; a record with several
shells is a MultiPolygon.  Test infrastructure only.
"""
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
US_STATES = os.path.join(HERE, "golden", "us_state", "cb_2017_us_state_20m")


def _signed_area2(r):
    return float(np.sum(r[:-1, 0] * r[1:, 1] - r[1:, 0] * r[:-1, 1]))


def read_shp_polygons(path):
    """-> list of polygons (list of parts, each a list of rings as (k, 2) float64 arrays, shell first)."""
    with open(path, "rb") as f:
        b = f.read()
    code, = struct.unpack_from(">i", b, 0)
    if code != 9994:
        raise ValueError("not a shapefile: %s" % path)
    o, polys = 100, []
    while o + 8 <= len(b):
        _, clen = struct.unpack_from(">ii", b, o)
        o += 8
        c = o
        o += 2 * clen
        st, = struct.unpack_from("<i", b, c)
        if st == 0:           # null shape
            polys.append([])
            continue
        if st not in (5, 15, 25):
            raise ValueError("shape type %d is not a polygon" % st)
        nparts, npts = struct.unpack_from("<ii", b, c + 36)
        parts = list(struct.unpack_from("<%di" % nparts, b, c + 44)) + [npts]
        xy = np.frombuffer(b, "<f8", 2 * npts, c + 44 + 4 * nparts).reshape(npts, 2).astype(np.float64)
        shells, holes = [], []
        for k in range(nparts):
            r = xy[parts[k]:parts[k + 1]]
            (shells if _signed_area2(r) <= 0 else holes).append(r)
        out = [[s] for s in shells]
        for h in holes:
            hx0, hy0 = h[:, 0].min(), h[:, 1].min()
            hx1, hy1 = h[:, 0].max(), h[:, 1].max()
            for part in out:
                s = part[0]
                if s[:, 0].min() <= hx0 and s[:, 1].min() <= hy0 and s[:, 0].max() >= hx1 and s[:, 1].max() >= hy1:
                    part.append(h)
                    break
            else:
                out.append([h[::-1]])   # an orphan hole is read as a shell
        polys.append(out)
    return polys


def read_dbf(path):
    """-> list of dicts (field name -> stripped string) of a dBASE III table."""
    with open(path, "rb") as f:
        b = f.read()
    nrec, hlen, rlen = struct.unpack_from("<IHH", b, 4)
    fields, o = [], 32
    while b[o] != 0x0D:
        name = b[o:o + 11].split(b"\0", 1)[0].decode("ascii")
        fields.append((name, b[o + 16]))
        o += 32
    rows = []
    for i in range(nrec):
        r = hlen + i * rlen + 1
        row = {}
        for name, ln in fields:
            row[name] = b[r:r + ln].decode("latin-1").strip()
            r += ln
        rows.append(row)
    return rows


def us_states():
    """(PolygonSet of the 52 records, their attribute rows)."""
    from geomesa_amd.join import PolygonSet
    return PolygonSet.from_polygons(read_shp_polygons(US_STATES + ".shp")), read_dbf(US_STATES + ".dbf")
