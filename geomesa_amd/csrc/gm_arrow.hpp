// gm_arrow.hpp -- device access to GeoMesa's Arrow geometry vectors (geomesa-arrow-jts): validity
// bits and ordinate tuples.  A tuple is [y, x] unless the vector's flipAxisOrder is set
// (AbstractPointVector.java:52-79, AbstractPolygonVector.java:72-79); Float4 vectors
// (PointFloatVector, ...FloatVector) widen their floats to double on read (readOrdinal).
#pragma once

#include "gm_internal.hpp"

namespace gm {

// Arrow validity bitmap, LSB bit order; NULL = every slot valid
__device__ __forceinline__ bool arrow_valid(const uint8_t* __restrict__ v, int64_t off, int64_t i) {
  if (!v) return true;
  const int64_t b = off + i;
  return (v[b >> 3] >> (b & 7)) & 1u;
}

// tuple j of an ordinate buffer -> (x, y)
template <bool F32>
__device__ __forceinline__ void arrow_tuple(const void* __restrict__ c, int64_t j, int flip, double& x, double& y) {
  double o0, o1;
  if (F32) {
    const float2 f = ((const float2*)c)[j];
    o0 = (double)f.x;
    o1 = (double)f.y;
  } else {
    const dv2 d = ((const dv2*)c)[j];
    o0 = d.x;
    o1 = d.y;
  }
  x = flip ? o0 : o1;
  y = flip ? o1 : o0;
}

// a point column as a kernel argument
struct ArrowPts {
  const void* c;
  const uint8_t* valid;
  int64_t voff;
  int32_t flip;
  int32_t f32;
};

}  // namespace gm
