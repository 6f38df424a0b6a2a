// gm_legacy.hip -- the deprecated curves GeoMesa keeps for reading and deleting old data:
// LegacyZ3SFC (curve/LegacyZ3SFC.scala:18-49), LegacyZ2SFC (LegacyZ2SFC.scala:14-26) and
// LegacyYearZ3SFC (LegacyYearZ3SFC.scala:17-46).  Same element-wise streaming shape as gm_curve.hip
// (the legacy indices Z3IndexV4/V6 and Z2IndexV3 only ever call index / invert per feature).
//
// SemiNormalizedDimension (NormalizedDimension.scala:83-87):
//   normalize(x)   = ceil((x - min) / (max - min) * precision).toInt
//   denormalize(i) = i == 0 ? min : (i - 0.5) * (max - min) / precision + min
// with precision 2^21-1 (lon, lat) and 2^20-1 (time) for Z3, 2^31-1 for Z2.  Legacy lenientIndex
// clamps only from below: max(dim.min, ceil(...)).toInt -- the bound is the dimension's *minimum
// coordinate* (-180 / -90 / 0), compared with the unclamped ceil, exactly as written.
#include "gm_keys.hpp"

namespace gm {

constexpr int LTPB = 256;

struct SemiDim {
  double min, max, prec;
};

__device__ __forceinline__ int32_t semi_normalize(const SemiDim& d, double x) {
  return jvm_d2i(ceil(((x - d.min) / (d.max - d.min)) * d.prec));
}
__device__ __forceinline__ int32_t semi_lenient(const SemiDim& d, double x) {
  const double c = ceil(((x - d.min) / (d.max - d.min)) * d.prec);
  return jvm_d2i(d.min >= c ? d.min : c);  // math.max(min, c); NaN c -> NaN -> 0
}
__device__ __forceinline__ double semi_denormalize(const SemiDim& d, int32_t i) {
  return i == 0 ? d.min : (((double)i - 0.5) * (d.max - d.min)) / d.prec + d.min;
}

__global__ __launch_bounds__(LTPB) void k_legacy_z3_index(const double* __restrict__ x, const double* __restrict__ y,
                                                          const int64_t* __restrict__ t, int64_t n, SemiDim lon,
                                                          SemiDim lat, SemiDim tim, int lenient,
                                                          int64_t* __restrict__ z, uint8_t* __restrict__ status,
                                                          int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * LTPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * LTPB) {
    const double xx = x[i], yy = y[i], td = (double)t[i];
    const bool inb = xx >= lon.min && xx <= lon.max && yy >= lat.min && yy <= lat.max && td >= tim.min &&
                     td <= tim.max;
    uint8_t st = ST_OK;
    int64_t zz = 0;
    if (inb) {
      zz = z3_apply(semi_normalize(lon, xx), semi_normalize(lat, yy), semi_normalize(tim, td));
    } else if (lenient) {  // LegacyZ3SFC.lenientIndex (LegacyZ3SFC.scala:23-28)
      zz = z3_apply(semi_lenient(lon, xx), semi_lenient(lat, yy), semi_lenient(tim, td));
    } else {
      st = ST_OUT_OF_BOUNDS;
    }
    z[i] = zz;
    if (status) status[i] = st;
    if (st) report_error(err, i, st);
  }
}

__global__ __launch_bounds__(LTPB) void k_legacy_z3_invert(const int64_t* __restrict__ z, int64_t n, SemiDim lon,
                                                           SemiDim lat, SemiDim tim, double* __restrict__ x,
                                                           double* __restrict__ y, int64_t* __restrict__ t) {
  for (int64_t i = (int64_t)blockIdx.x * LTPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * LTPB) {
    const int64_t zz = z[i];
    x[i] = semi_denormalize(lon, z3_combine(zz));
    y[i] = semi_denormalize(lat, z3_combine(zz >> 1));
    t[i] = jvm_d2l(semi_denormalize(tim, z3_combine(zz >> 2)));
  }
}

__global__ __launch_bounds__(LTPB) void k_legacy_z2_index(const double* __restrict__ x, const double* __restrict__ y,
                                                          int64_t n, SemiDim lon, SemiDim lat, int lenient,
                                                          int64_t* __restrict__ z, uint8_t* __restrict__ status,
                                                          int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * LTPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * LTPB) {
    const double xx = x[i], yy = y[i];
    const bool inb = xx >= lon.min && xx <= lon.max && yy >= lat.min && yy <= lat.max;
    uint8_t st = ST_OK;
    int64_t zz = 0;
    if (inb) zz = z2_apply(semi_normalize(lon, xx), semi_normalize(lat, yy));
    else if (lenient) zz = z2_apply(semi_lenient(lon, xx), semi_lenient(lat, yy));  // LegacyZ2SFC.scala:20-24
    else st = ST_OUT_OF_BOUNDS;
    z[i] = zz;
    if (status) status[i] = st;
    if (st) report_error(err, i, st);
  }
}

__global__ __launch_bounds__(LTPB) void k_legacy_z2_invert(const int64_t* __restrict__ z, int64_t n, SemiDim lon,
                                                           SemiDim lat, double* __restrict__ x,
                                                           double* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * LTPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * LTPB) {
    const int64_t zz = z[i];
    x[i] = semi_denormalize(lon, z2_combine(zz));
    y[i] = semi_denormalize(lat, z2_combine(zz >> 1));
  }
}

// LegacyYearZ3SFC.index (LegacyYearZ3SFC.scala:24-30): the standard 21-bit curve with the legacy
// (too short) time max of 52 weeks in minutes; offsets in (52 weeks, maxOffset(Year)] index as the max
template <bool LENIENT>
__global__ __launch_bounds__(LTPB) void k_legacy_year_z3_index(const double* __restrict__ x,
                                                               const double* __restrict__ y,
                                                               const int64_t* __restrict__ t, int64_t n, NDim lon,
                                                               NDim lat, NDim tim, int64_t year_max,
                                                               int64_t* __restrict__ z, uint8_t* __restrict__ status,
                                                               int64_t* __restrict__ err) {
  const int64_t tmax = (int64_t)tim.max;  // time.max.toLong
  for (int64_t i = (int64_t)blockIdx.x * LTPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * LTPB) {
    int64_t tt = t[i];
    if ((double)tt > tim.max && tt <= year_max) tt = tmax;
    int64_t zz;
    const uint8_t st = z3_index_one<LENIENT>(x[i], y[i], tt, lon, lat, tim, zz);
    z[i] = zz;
    if (status) status[i] = st;
    if (st) report_error(err, i, st);
  }
}

inline unsigned legacy_grid(int64_t n) {
  int64_t g = (n + LTPB - 1) / LTPB;
  if (g > 256 * 32) g = 256 * 32;
  return (unsigned)(g < 1 ? 1 : g);
}

inline SemiDim semi(double mn, double mx, int64_t prec) { return SemiDim{mn, mx, (double)prec}; }

}  // namespace gm

using namespace gm;

extern "C" {

int gm_legacy_z3_index(gm_ctx* ctx, const double* x, const double* y, const int64_t* t, int64_t n, int curve,
                       int period, int lenient, int64_t* z, uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || !valid_period(period) || (curve != GM_LEGACY_Z3 && curve != GM_LEGACY_YEAR_Z3))
    return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!x || !y || !t || !z) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  if (curve == GM_LEGACY_Z3) {
    // LegacyZ3Dimensions (LegacyZ3SFC.scala:43-48)
    const SemiDim lon = semi(-180.0, 180.0, (1 << 21) - 1), lat = semi(-90.0, 90.0, (1 << 21) - 1);
    const SemiDim tim = semi(0.0, (double)max_offset(period), (1 << 20) - 1);
    hipLaunchKernelGGL(k_legacy_z3_index, dim3(legacy_grid(n)), dim3(LTPB), 0, ctx->stream, x, y, t, n, lon, lat,
                       tim, lenient, z, status, ctx->d_err);
  } else {
    // LegacyYearZ3Dimensions (LegacyYearZ3SFC.scala:38-45): NormalizedTime(21, 52 weeks in minutes)
    const NDim lon = lon_dim(21), lat = lat_dim(21), tim = make_ndim(0.0, 7.0 * 24 * 60 * 52, 21);
    const int64_t ymax = max_offset(YEAR);
    if (lenient)
      hipLaunchKernelGGL((k_legacy_year_z3_index<true>), dim3(legacy_grid(n)), dim3(LTPB), 0, ctx->stream, x, y, t,
                         n, lon, lat, tim, ymax, z, status, ctx->d_err);
    else
      hipLaunchKernelGGL((k_legacy_year_z3_index<false>), dim3(legacy_grid(n)), dim3(LTPB), 0, ctx->stream, x, y,
                         t, n, lon, lat, tim, ymax, z, status, ctx->d_err);
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_legacy_z3_invert(gm_ctx* ctx, const int64_t* z, int64_t n, int curve, int period, double* x, double* y,
                        int64_t* t) {
  if (!ctx || n < 0 || !valid_period(period) || curve != GM_LEGACY_Z3) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!z || !x || !y || !t) return GM_E_INVALID;
  const SemiDim lon = semi(-180.0, 180.0, (1 << 21) - 1), lat = semi(-90.0, 90.0, (1 << 21) - 1);
  const SemiDim tim = semi(0.0, (double)max_offset(period), (1 << 20) - 1);
  hipLaunchKernelGGL(k_legacy_z3_invert, dim3(legacy_grid(n)), dim3(LTPB), 0, ctx->stream, z, n, lon, lat, tim, x,
                     y, t);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

int gm_legacy_z2_index(gm_ctx* ctx, const double* x, const double* y, int64_t n, int lenient, int64_t* z,
                       uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!x || !y || !z) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const SemiDim lon = semi(-180.0, 180.0, 2147483647LL), lat = semi(-90.0, 90.0, 2147483647LL);
  hipLaunchKernelGGL(k_legacy_z2_index, dim3(legacy_grid(n)), dim3(LTPB), 0, ctx->stream, x, y, n, lon, lat, lenient,
                     z, status, ctx->d_err);
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_legacy_z2_invert(gm_ctx* ctx, const int64_t* z, int64_t n, double* x, double* y) {
  if (!ctx || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!z || !x || !y) return GM_E_INVALID;
  const SemiDim lon = semi(-180.0, 180.0, 2147483647LL), lat = semi(-90.0, 90.0, 2147483647LL);
  hipLaunchKernelGGL(k_legacy_z2_invert, dim3(legacy_grid(n)), dim3(LTPB), 0, ctx->stream, z, n, lon, lat, x, y);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

}  // extern "C"
