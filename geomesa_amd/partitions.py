"""geomesa-fs spatial partition schemes: Z2Scheme / XZ2Scheme.

Mirrors geomesa-fs-storage-common/.../partitions/{SpatialScheme,Z2Scheme,XZ2Scheme}.scala: the
partition name of a feature is its Z2 (Z2SFC(bits / 2)) or XZ2 (XZ2SFC(bits / 2)) index, zero-padded
to `digits(bits)` decimal places (SpatialScheme.scala:25; Z2Scheme.scala:50, XZ2Scheme.scala:28).
Names for a batch of features come from the gm_z2_index / gm_xz2_index kernels (non-lenient, as
`z2.index(pt.getX, pt.getY)` and `xz2.index(env...)` throw on out-of-bounds input); the bbox query
side enumerates every index inside the curve's ranges (SpatialScheme.getIntersectingPartitions
:43-56) on the host, as the reference does.
"""
import math

import numpy as np

from .curve import IllegalArgumentException, XZ2SFC, Z2SFC


class SpatialScheme:
    name = None

    def __init__(self, bits, geom="geom"):
        if bits % 2 != 0:   # SpatialScheme.scala:23
            raise IllegalArgumentException("Resolution must be an even number")
        self.bits, self.geom = int(bits), geom
        self.format = "%%0%dd" % self.digits(self.bits)

    @property
    def pattern(self):
        return "%d-bit-%s" % (self.bits, self.name)

    def _names(self, idx):
        a = idx.cpu().numpy() if hasattr(idx, "cpu") else np.asarray(idx)
        return [self.format % int(v) for v in a]

    def intersecting_partitions(self, boxes):
        """getIntersectingPartitions for bbox filters (xmin, ymin, xmax, ymax) OR'd together; an empty list
        of boxes is the 'no spatial filter' case (None)."""
        if not boxes:
            return None
        seen, out = set(), []
        for r in self.generate_ranges([tuple(map(float, b)) for b in boxes]):
            for v in range(int(r.lower), int(r.upper) + 1):
                if v not in seen:
                    seen.add(v)
                    out.append(self.format % v)
        return out


class Z2Scheme(SpatialScheme):
    """Z2Scheme(bits, geom) (Z2Scheme.scala:19-52): point geometries only."""
    name = "z2"

    def __init__(self, bits, geom="geom"):
        super().__init__(bits, geom)
        self.z2 = Z2SFC(self.bits // 2)
        self.x_radius = (360.0 / math.pow(2, self.bits // 2)) / 2
        self.y_radius = (180.0 / math.pow(2, self.bits // 2)) / 2

    @staticmethod
    def digits(bits):   # Z2Scheme.scala:50
        return int(math.ceil(bits * math.log10(2)))

    def partition_names(self, x, y):
        """getPartitionName for a batch of points (Z2Scheme.scala:26-29)."""
        return self._names(self.z2.index(x, y))

    def generate_ranges(self, xy):
        return self.z2.ranges(xy)

    def covering_bounds(self, partition):
        """getCoveringFilter (Z2Scheme.scala:31-45) as (xmin, ymin, xmax, ymax, x_exclusive, y_exclusive):
        the cell's bbox, with the upper bounds exclusive except on the world's upper-right edge."""
        x, y = self.z2.invert([int(partition)])
        x, y = float(x[0]), float(y[0])
        xmin, xmax = x - self.x_radius, x + self.x_radius
        ymin, ymax = y - self.y_radius, y + self.y_radius
        return xmin, ymin, xmax, ymax, xmax != self.z2.lon.max, ymax != self.z2.lat.max


class XZ2Scheme(SpatialScheme):
    """XZ2Scheme(bits, geom) (XZ2Scheme.scala:11-31): any geometry, by its envelope."""
    name = "xz2"

    def __init__(self, bits, geom="geom"):
        super().__init__(bits, geom)
        self.xz2 = XZ2SFC(self.bits // 2)

    @staticmethod
    def digits(bits):   # XZ2Scheme.scala:27-28: digits of the largest sequence code
        return int(math.ceil(((bits // 2) + 1) * math.log10(4) - math.log10(3)))

    def partition_names(self, xmin, ymin, xmax=None, ymax=None):
        """getPartitionName for a batch of envelopes (points: xmax/ymax omitted) (XZ2Scheme.scala:16-20)."""
        if xmax is None:
            xmax, ymax = xmin, ymin
        return self._names(self.xz2.index(xmin, ymin, xmax, ymax))

    def generate_ranges(self, xy):
        return self.xz2.ranges(xy)


__all__ = ["SpatialScheme", "Z2Scheme", "XZ2Scheme"]
