"""geomesa_amd -- MI355X-native (gfx950 HIP) GeoMesa spatio-temporal index-and-filter hot path.

Host-side mirror of the reference Scala API for the hot path (Z3SFC/Z2SFC/XZ2SFC/XZ3SFC,
Z3Filter/Z2Filter, Z3IndexKeySpace planning, st_contains join) over the C-ABI library
libgeomesa_hip.so (include/geomesa_hip.h).  All per-row compute runs in the HIP library.
"""
from .curve import (BinnedTime, CoveredRange, IllegalArgumentException, IndexRange, OverlappingRange,  # noqa: F401
                    TimePeriod, XZ2SFC, XZ3SFC, Z2SFC, Z3SFC)

__version__ = "0.1.0"
