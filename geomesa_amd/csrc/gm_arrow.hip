// gm_arrow.hip -- index keys straight from GeoMesa's Arrow geometry vectors.
//
// The JVM side of GeoMesa already holds feature batches as Arrow vectors (geomesa-arrow-jts); these
// entry points read them in place: no per-feature JTS objects and no de-interleaving copy.
//   * point keys (Z3 / Z2): pair layout as the column kernels -- lane l of a wave step takes the
//     tuples 2p and 2p+1 (32 contiguous bytes of Float8 ordinates), the date pair as one 16-B load,
//     and stores z / bin pairs with one 16-B / 4-B store; validity bits are read per row (one byte
//     covers 8 rows, L1-resident);
//   * envelope keys (XZ2 / XZ3): one geometry per lane, walking its List offsets and tuples with the
//     JTS envelope rules (Geometry.getEnvelopeInternal), then the same XZ code as gm_xz2_index;
//   * gm_arrow_points_to_columns: the x / y adapter for every other entry (null -> NaN).
#include <algorithm>
#include <vector>

#include "gm_arrow.hpp"
#include "gm_keys.hpp"

namespace gm {

constexpr int ATPB = 256;

struct ArrowTime {
  const int64_t* ms;
  const uint8_t* valid;
  int64_t voff;
};

// the feature's date: a null column or a null slot is time 0 (Z3IndexKeySpace.scala:70-71)
__device__ __forceinline__ int64_t arrow_time(const ArrowTime& t, int64_t i) {
  if (!t.ms || !arrow_valid(t.valid, t.voff, i)) return 0;
  return t.ms[i];
}

__device__ __forceinline__ void arrow_time_pair(const ArrowTime& t, int64_t p, bool vec, int64_t& t0, int64_t& t1) {
  if (!t.ms) { t0 = t1 = 0; return; }
  if (vec) {
    const lv2 v = __builtin_nontemporal_load(&((const lv2*)t.ms)[p]);
    t0 = v.x; t1 = v.y;
  } else {
    t0 = t.ms[2 * p]; t1 = t.ms[2 * p + 1];
  }
  if (!arrow_valid(t.valid, t.voff, 2 * p)) t0 = 0;
  if (!arrow_valid(t.valid, t.voff, 2 * p + 1)) t1 = 0;
}

// ------------------------------------------------------------------ Z3 / Z2 point keys

template <int PERIOD, bool LENIENT, bool F32, bool VEC>
__global__ __launch_bounds__(ATPB) void k_z3_key_arrow(ArrowPts g, ArrowTime tc, int64_t n, NDim lon, NDim lat,
                                                       NDim tim, int16_t* __restrict__ bin, int64_t* __restrict__ z,
                                                       uint8_t* __restrict__ status, int64_t* __restrict__ err) {
  const int64_t npairs = (n + 1) >> 1;
  for (int64_t p = (int64_t)blockIdx.x * ATPB + threadIdx.x; p < npairs; p += (int64_t)gridDim.x * ATPB) {
    const bool two = 2 * p + 1 < n;
    int16_t b[2] = {0, 0};
    int64_t zz[2] = {0, 0};
    uint8_t st[2] = {ST_OK, ST_OK};
    int64_t tt[2];
    if (two) arrow_time_pair(tc, p, VEC, tt[0], tt[1]);
    else { tt[0] = arrow_time(tc, 2 * p); tt[1] = 0; }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t i = 2 * p + j;
      if (j == 1 && !two) break;
      if (!arrow_valid(g.valid, g.voff, i)) { st[j] = ST_NULL_GEOM; continue; }
      double x, y;
      arrow_tuple<F32>(g.c, i, g.flip, x, y);
      st[j] = z3_key_one<PERIOD, LENIENT>(x, y, tt[j], lon, lat, tim, b[j], zz[j]);
    }
    if (VEC && two) {
      st_stream(lv2{zz[0], zz[1]}, &((lv2*)z)[p]);
      ((short2*)bin)[p] = make_short2(b[0], b[1]);
      if (status) ((uchar2*)status)[p] = make_uchar2(st[0], st[1]);
    } else {
      z[2 * p] = zz[0]; bin[2 * p] = b[0];
      if (status) status[2 * p] = st[0];
      if (two) { z[2 * p + 1] = zz[1]; bin[2 * p + 1] = b[1]; if (status) status[2 * p + 1] = st[1]; }
    }
    if (st[0]) report_error(err, 2 * p, st[0]);
    if (two && st[1]) report_error(err, 2 * p + 1, st[1]);
  }
}

// the aligned, full-pair form of k_z3_key_arrow: one chunk of ATPB * UNROLL pairs per workgroup, every
// load of the chunk issued before any compute (as k_z3_index_key): tuples 2p, 2p+1 as two 16-B loads
// (Float8) or one (Float4), the date pair as one 16-B load
template <bool F32>
__device__ __forceinline__ void arrow_tuple_pair(const void* __restrict__ c, int64_t p, dv2& a, dv2& b) {
  if (F32) {
    typedef float fv4 __attribute__((ext_vector_type(4)));
    const fv4 f = __builtin_nontemporal_load(&((const fv4*)c)[p]);
    a = dv2{(double)f.x, (double)f.y};
    b = dv2{(double)f.z, (double)f.w};
  } else {
    a = __builtin_nontemporal_load(&((const dv2*)c)[2 * p]);
    b = __builtin_nontemporal_load(&((const dv2*)c)[2 * p + 1]);
  }
}

template <int PERIOD, bool LENIENT, bool F32, bool TIME, int UNROLL>
__global__ __launch_bounds__(ATPB) void k_z3_key_arrow_v(ArrowPts g, ArrowTime tc, int64_t n, NDim lon, NDim lat,
                                                         NDim tim, short2* __restrict__ bin, lv2* __restrict__ z,
                                                         uchar2* __restrict__ status, int64_t* __restrict__ err) {
  static_assert(UNROLL == 4, "staged bins: 4 pairs per lane");
  __shared__ uint32_t s_bin[ATPB * UNROLL];   // the block's bins, stored 16 B per lane at the end
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (ATPB * UNROLL) + threadIdx.x;
  dv2 a[UNROLL], b[UNROLL];
  lv2 tv[UNROLL];
  if (((int64_t)blockIdx.x + 1) * (ATPB * UNROLL) <= npairs) {
    // a full block: every load unconditional, so all 2-3 x UNROLL are in flight before the first wait
    // (the guarded form below is waited for pair by pair: see ld_stream, gm_keys.hpp)
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t p = base + (int64_t)u * ATPB;
      arrow_tuple_pair<F32>(g.c, p, a[u], b[u]);
      tv[u] = TIME ? __builtin_nontemporal_load(&((const lv2*)tc.ms)[p]) : lv2{0, 0};
    }
  } else {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t p = base + (int64_t)u * ATPB;
      tv[u] = lv2{0, 0};
      if (p < npairs) {
        arrow_tuple_pair<F32>(g.c, p, a[u], b[u]);
        if (TIME) tv[u] = __builtin_nontemporal_load(&((const lv2*)tc.ms)[p]);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * ATPB;
    if (p >= npairs) continue;
    if (TIME && tc.valid) {
      if (!arrow_valid(tc.valid, tc.voff, 2 * p)) tv[u].x = 0;
      if (!arrow_valid(tc.valid, tc.voff, 2 * p + 1)) tv[u].y = 0;
    }
    int16_t b0 = 0, b1 = 0;
    int64_t z0 = 0, z1 = 0;
    const double x0 = g.flip ? a[u].x : a[u].y, y0 = g.flip ? a[u].y : a[u].x;
    const double x1 = g.flip ? b[u].x : b[u].y, y1 = g.flip ? b[u].y : b[u].x;
    uint8_t s0 = ST_NULL_GEOM, s1 = ST_NULL_GEOM;
    if (arrow_valid(g.valid, g.voff, 2 * p)) s0 = z3_key_one<PERIOD, LENIENT>(x0, y0, tv[u].x, lon, lat, tim, b0, z0);
    if (arrow_valid(g.valid, g.voff, 2 * p + 1)) s1 = z3_key_one<PERIOD, LENIENT>(x1, y1, tv[u].y, lon, lat, tim, b1, z1);
    st_stream(lv2{z0, z1}, &z[p]);
    s_bin[u * ATPB + threadIdx.x] = bin_pair(b0, b1);
    if (status) status[p] = make_uchar2(s0, s1);
    if (s0) report_error(err, 2 * p, s0);
    if (s1) report_error(err, 2 * p + 1, s1);
  }
  store_staged_bins<ATPB>(s_bin, bin, npairs);
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {   // the odd last row
    const int64_t i = n - 1;
    int16_t bb = 0;
    int64_t zz = 0;
    uint8_t st = ST_NULL_GEOM;
    if (arrow_valid(g.valid, g.voff, i)) {
      double x, y;
      arrow_tuple<F32>(g.c, i, g.flip, x, y);
      st = z3_key_one<PERIOD, LENIENT>(x, y, TIME ? arrow_time(tc, i) : 0, lon, lat, tim, bb, zz);
    }
    ((int16_t*)bin)[i] = bb;
    ((int64_t*)z)[i] = zz;
    if (status) ((uint8_t*)status)[i] = st;
    if (st) report_error(err, i, st);
  }
}

template <bool LENIENT, bool F32, bool VEC>
__global__ __launch_bounds__(ATPB) void k_z2_key_arrow(ArrowPts g, int64_t n, NDim lon, NDim lat,
                                                       int64_t* __restrict__ z, uint8_t* __restrict__ status,
                                                       int64_t* __restrict__ err) {
  const int64_t npairs = (n + 1) >> 1;
  for (int64_t p = (int64_t)blockIdx.x * ATPB + threadIdx.x; p < npairs; p += (int64_t)gridDim.x * ATPB) {
    const bool two = 2 * p + 1 < n;
    int64_t zz[2] = {0, 0};
    uint8_t st[2] = {ST_OK, ST_OK};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t i = 2 * p + j;
      if (j == 1 && !two) break;
      if (!arrow_valid(g.valid, g.voff, i)) { st[j] = ST_NULL_GEOM; continue; }
      double x, y;
      arrow_tuple<F32>(g.c, i, g.flip, x, y);
      st[j] = z2_index_one<LENIENT>(x, y, lon, lat, zz[j]);
    }
    if (VEC && two) {
      st_stream(lv2{zz[0], zz[1]}, &((lv2*)z)[p]);
      if (status) ((uchar2*)status)[p] = make_uchar2(st[0], st[1]);
    } else {
      z[2 * p] = zz[0];
      if (status) status[2 * p] = st[0];
      if (two) { z[2 * p + 1] = zz[1]; if (status) status[2 * p + 1] = st[1]; }
    }
    if (st[0]) report_error(err, 2 * p, st[0]);
    if (two && st[1]) report_error(err, 2 * p + 1, st[1]);
  }
}

template <bool F32>
__global__ __launch_bounds__(ATPB) void k_points_soa(ArrowPts g, int64_t n, double* __restrict__ x,
                                                     double* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * ATPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * ATPB) {
    double px = NAN, py = NAN;
    if (arrow_valid(g.valid, g.voff, i)) arrow_tuple<F32>(g.c, i, g.flip, px, py);
    x[i] = px;
    y[i] = py;
  }
}

// ------------------------------------------------------------------ envelopes (XZ keys)
// org.locationtech.jts.geom.Envelope: expandToInclude(x, y) initialises a null envelope and
// otherwise widens with strict compares (a NaN ordinate never widens); expandToInclude(Envelope)
// skips a null envelope.  The null envelope reads back as (minx 0, maxx -1, miny 0, maxy -1).
struct Env {
  double minx, maxx, miny, maxy;
  bool null_;
};

__device__ __forceinline__ Env env_null() { return Env{0.0, -1.0, 0.0, -1.0, true}; }

__device__ __forceinline__ void env_expand(Env& e, double x, double y) {
  if (e.null_) { e = Env{x, x, y, y, false}; return; }
  if (x < e.minx) e.minx = x;
  if (x > e.maxx) e.maxx = x;
  if (y < e.miny) e.miny = y;
  if (y > e.maxy) e.maxy = y;
}

__device__ __forceinline__ void env_merge(Env& e, const Env& o) {
  if (o.null_) return;
  if (e.null_) { e = o; return; }
  if (o.minx < e.minx) e.minx = o.minx;
  if (o.maxx > e.maxx) e.maxx = o.maxx;
  if (o.miny < e.miny) e.miny = o.miny;
  if (o.maxy > e.maxy) e.maxy = o.maxy;
}

struct ArrowGeom {
  const void* c;
  const uint8_t* valid;
  int64_t voff;
  const int32_t* o0;
  const int32_t* o1;
  const int32_t* o2;
  int32_t type;
  int32_t flip;
};

// CoordinateSequence.expandEnvelope over tuples [a, b)
template <bool F32>
__device__ __forceinline__ Env env_tuples(const ArrowGeom& g, int64_t a, int64_t b) {
  Env e = env_null();
  for (int64_t j = a; j < b; ++j) {
    double x, y;
    arrow_tuple<F32>(g.c, j, g.flip, x, y);
    env_expand(e, x, y);
  }
  return e;
}

// Geometry.getEnvelopeInternal of slot i: a polygon's is its shell's (Polygon.computeEnvelopeInternal),
// a multi geometry's the merge of its parts' (GeometryCollection.computeEnvelopeInternal)
template <bool F32>
__device__ Env geom_envelope(const ArrowGeom& g, int64_t i) {
  switch (g.type) {
    case GM_GEOM_POINT: {
      Env e = env_null();
      double x, y;
      arrow_tuple<F32>(g.c, i, g.flip, x, y);
      env_expand(e, x, y);
      return e;
    }
    case GM_GEOM_LINESTRING:
    case GM_GEOM_MULTIPOINT:
      return env_tuples<F32>(g, g.o0[i], g.o0[i + 1]);
    case GM_GEOM_POLYGON: {
      const int32_t r0 = g.o0[i], r1 = g.o0[i + 1];
      if (r1 <= r0) return env_null();
      return env_tuples<F32>(g, g.o1[r0], g.o1[r0 + 1]);
    }
    case GM_GEOM_MULTILINESTRING: {
      Env e = env_null();
      for (int32_t l = g.o0[i]; l < g.o0[i + 1]; ++l) env_merge(e, env_tuples<F32>(g, g.o1[l], g.o1[l + 1]));
      return e;
    }
    default: {   // GM_GEOM_MULTIPOLYGON
      Env e = env_null();
      for (int32_t p = g.o0[i]; p < g.o0[i + 1]; ++p) {
        const int32_t r0 = g.o1[p], r1 = g.o1[p + 1];
        if (r1 > r0) env_merge(e, env_tuples<F32>(g, g.o2[r0], g.o2[r0 + 1]));
      }
      return e;
    }
  }
}

// XZ2IndexKeySpace / XZ3IndexKeySpace.toIndexKey over an Arrow geometry column; DIM 3 also bins the date
template <int DIM, int PERIOD, bool LENIENT, bool F32>
__global__ __launch_bounds__(ATPB) void k_xz_key_arrow(ArrowGeom g, ArrowTime tc, int64_t n, int gp, double zhi,
                                                       int16_t* __restrict__ bin, int64_t* __restrict__ xz,
                                                       uint8_t* __restrict__ status, int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * ATPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * ATPB) {
    int64_t out = 0;
    int16_t b = 0;
    uint8_t st;
    if (!arrow_valid(g.valid, g.voff, i)) {
      st = ST_NULL_GEOM;
    } else {
      const Env e = geom_envelope<F32>(g, i);
      if (DIM == 2) {
        st = xz2_one<LENIENT>(gp, e.minx, e.miny, e.maxx, e.maxy, out);
      } else {
        int64_t off;
        st = binned_time<PERIOD>(arrow_time(tc, i), b, off);   // outside the try: throws even when lenient
        if (st == ST_OK) {
          const double t = (double)off;
          st = xz3_one<LENIENT>(gp, zhi, e.minx, e.miny, t, e.maxx, e.maxy, t, out);
        }
        if (st != ST_OK) b = 0;
      }
    }
    if (st != ST_OK) out = 0;
    xz[i] = out;
    if (DIM == 3) bin[i] = b;
    if (status) status[i] = st;
    if (st) report_error(err, i, st);
  }
}

// ------------------------------------------------------------------ host side

inline unsigned agrid(int64_t units) {
  int64_t b = (units + ATPB - 1) / ATPB;
  if (b > 256 * 32) b = 256 * 32;
  return (unsigned)(b < 1 ? 1 : b);
}

inline bool point_col_ok(const gm_geom_column* g) {
  return g && g->type == GM_GEOM_POINT && (g->ordinal_bits == 64 || g->ordinal_bits == 32) && g->coords;
}

inline ArrowPts to_pts(const gm_geom_column* g) {
  return ArrowPts{g->coords, g->validity, g->validity_offset, g->flip_axis, g->ordinal_bits == 32};
}

inline ArrowTime to_time(const gm_time_column* t) {
  return t ? ArrowTime{t->millis, t->validity, t->validity_offset} : ArrowTime{nullptr, nullptr, 0};
}

constexpr int AUNROLL = 4;

template <int PERIOD, bool LENIENT, bool F32>
void launch_z3_arrow(hipStream_t s, bool vec, ArrowPts g, ArrowTime tc, int64_t n, NDim lon, NDim lat, NDim tim,
                     int16_t* bin, int64_t* z, uint8_t* status, int64_t* err) {
  if (vec && aligned16(g.c) && n >= 2) {
    const int64_t np = n >> 1;
    const unsigned vg = (unsigned)((np + ATPB * AUNROLL - 1) / (ATPB * AUNROLL));
    if (tc.ms)
      hipLaunchKernelGGL((k_z3_key_arrow_v<PERIOD, LENIENT, F32, true, AUNROLL>), dim3(vg), dim3(ATPB), 0, s, g, tc, n,
                         lon, lat, tim, (short2*)bin, (lv2*)z, (uchar2*)status, err);
    else
      hipLaunchKernelGGL((k_z3_key_arrow_v<PERIOD, LENIENT, F32, false, AUNROLL>), dim3(vg), dim3(ATPB), 0, s, g, tc, n,
                         lon, lat, tim, (short2*)bin, (lv2*)z, (uchar2*)status, err);
    return;
  }
  const unsigned grid = agrid((n + 1) >> 1);
  if (vec) hipLaunchKernelGGL((k_z3_key_arrow<PERIOD, LENIENT, F32, true>), dim3(grid), dim3(ATPB), 0, s, g, tc, n, lon, lat, tim, bin, z, status, err);
  else hipLaunchKernelGGL((k_z3_key_arrow<PERIOD, LENIENT, F32, false>), dim3(grid), dim3(ATPB), 0, s, g, tc, n, lon, lat, tim, bin, z, status, err);
}

template <int PERIOD>
void launch_z3_arrow_p(hipStream_t s, bool vec, bool lenient, bool f32, ArrowPts g, ArrowTime tc, int64_t n, NDim lon,
                       NDim lat, NDim tim, int16_t* bin, int64_t* z, uint8_t* status, int64_t* err) {
  if (lenient) {
    if (f32) launch_z3_arrow<PERIOD, true, true>(s, vec, g, tc, n, lon, lat, tim, bin, z, status, err);
    else launch_z3_arrow<PERIOD, true, false>(s, vec, g, tc, n, lon, lat, tim, bin, z, status, err);
  } else {
    if (f32) launch_z3_arrow<PERIOD, false, true>(s, vec, g, tc, n, lon, lat, tim, bin, z, status, err);
    else launch_z3_arrow<PERIOD, false, false>(s, vec, g, tc, n, lon, lat, tim, bin, z, status, err);
  }
}

template <int DIM, int PERIOD>
void launch_xz_arrow(hipStream_t s, bool lenient, bool f32, ArrowGeom g, ArrowTime tc, int64_t n, int gp, double zhi,
                     int16_t* bin, int64_t* xz, uint8_t* status, int64_t* err) {
  const unsigned grid = agrid(n);
  if (lenient) {
    if (f32) hipLaunchKernelGGL((k_xz_key_arrow<DIM, PERIOD, true, true>), dim3(grid), dim3(ATPB), 0, s, g, tc, n, gp, zhi, bin, xz, status, err);
    else hipLaunchKernelGGL((k_xz_key_arrow<DIM, PERIOD, true, false>), dim3(grid), dim3(ATPB), 0, s, g, tc, n, gp, zhi, bin, xz, status, err);
  } else {
    if (f32) hipLaunchKernelGGL((k_xz_key_arrow<DIM, PERIOD, false, true>), dim3(grid), dim3(ATPB), 0, s, g, tc, n, gp, zhi, bin, xz, status, err);
    else hipLaunchKernelGGL((k_xz_key_arrow<DIM, PERIOD, false, false>), dim3(grid), dim3(ATPB), 0, s, g, tc, n, gp, zhi, bin, xz, status, err);
  }
}

// the List offsets a geometry type needs, outermost first
inline int offset_levels(int type) {
  switch (type) {
    case GM_GEOM_POINT: return 0;
    case GM_GEOM_LINESTRING: case GM_GEOM_MULTIPOINT: return 1;
    case GM_GEOM_POLYGON: case GM_GEOM_MULTILINESTRING: return 2;
    case GM_GEOM_MULTIPOLYGON: return 3;
    default: return -1;
  }
}

inline bool geom_col_ok(const gm_geom_column* g) {
  if (!g || !g->coords || (g->ordinal_bits != 64 && g->ordinal_bits != 32)) return false;
  const int lv = offset_levels(g->type);
  if (lv < 0) return false;
  for (int k = 0; k < lv; ++k)
    if (!g->offsets[k]) return false;
  return true;
}

}  // namespace gm

using namespace gm;

extern "C" {

int gm_z3_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, const gm_time_column* dtg, int64_t n, int period,
                          int lenient, int16_t* bin, int64_t* z, uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || !valid_period(period)) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!point_col_ok(geom) || !bin || !z) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const NDim lon = lon_dim(21), lat = lat_dim(21), tim = time_dim(period, 21);
  const ArrowTime tc = to_time(dtg);
  const bool vec = aligned16(z) && (((uintptr_t)bin & 3u) == 0) && (((uintptr_t)status & 1u) == 0) &&
                   (!tc.ms || aligned16(tc.ms));
  const bool f32 = geom->ordinal_bits == 32;
  const ArrowPts g = to_pts(geom);
  hipStream_t s = ctx->stream;
  switch (period) {
    case DAY: launch_z3_arrow_p<DAY>(s, vec, lenient, f32, g, tc, n, lon, lat, tim, bin, z, status, ctx->d_err); break;
    case WEEK: launch_z3_arrow_p<WEEK>(s, vec, lenient, f32, g, tc, n, lon, lat, tim, bin, z, status, ctx->d_err); break;
    case MONTH: launch_z3_arrow_p<MONTH>(s, vec, lenient, f32, g, tc, n, lon, lat, tim, bin, z, status, ctx->d_err); break;
    default: launch_z3_arrow_p<YEAR>(s, vec, lenient, f32, g, tc, n, lon, lat, tim, bin, z, status, ctx->d_err); break;
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_z2_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, int64_t n, int lenient, int64_t* z, uint8_t* status,
                          gm_batch_status* summary) {
  if (!ctx || n < 0) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!point_col_ok(geom) || !z) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const NDim lon = lon_dim(31), lat = lat_dim(31);   // Z2SFC object: 31 bits per dimension
  const bool vec = aligned16(z) && (((uintptr_t)status & 1u) == 0);
  const ArrowPts g = to_pts(geom);
  const unsigned grid = agrid((n + 1) >> 1);
  hipStream_t s = ctx->stream;
  int64_t* err = ctx->d_err;
  const bool f32 = geom->ordinal_bits == 32;
#define GM_Z2A(L, F, V) hipLaunchKernelGGL((k_z2_key_arrow<L, F, V>), dim3(grid), dim3(ATPB), 0, s, g, n, lon, lat, z, status, err)
  if (lenient) {
    if (f32) { if (vec) GM_Z2A(true, true, true); else GM_Z2A(true, true, false); }
    else { if (vec) GM_Z2A(true, false, true); else GM_Z2A(true, false, false); }
  } else {
    if (f32) { if (vec) GM_Z2A(false, true, true); else GM_Z2A(false, true, false); }
    else { if (vec) GM_Z2A(false, false, true); else GM_Z2A(false, false, false); }
  }
#undef GM_Z2A
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

static int xz_key_arrow(gm_ctx* ctx, int dim, const gm_geom_column* geom, const gm_time_column* dtg, int64_t n, int g,
                        int period, int lenient, int16_t* bin, int64_t* xz, uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || g < 1 || g > (dim == 2 ? 30 : 20) || (dim == 3 && !valid_period(period))) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!geom_col_ok(geom) || !xz || (dim == 3 && !bin)) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const ArrowGeom ag{geom->coords, geom->validity, geom->validity_offset, geom->offsets[0], geom->offsets[1],
                     geom->offsets[2], geom->type, geom->flip_axis};
  const ArrowTime tc = to_time(dtg);
  const bool f32 = geom->ordinal_bits == 32;
  hipStream_t s = ctx->stream;
  if (dim == 2) {
    launch_xz_arrow<2, WEEK>(s, lenient, f32, ag, tc, n, g, 0.0, bin, xz, status, ctx->d_err);
  } else {
    const double zhi = (double)max_offset(period);
    switch (period) {
      case DAY: launch_xz_arrow<3, DAY>(s, lenient, f32, ag, tc, n, g, zhi, bin, xz, status, ctx->d_err); break;
      case WEEK: launch_xz_arrow<3, WEEK>(s, lenient, f32, ag, tc, n, g, zhi, bin, xz, status, ctx->d_err); break;
      case MONTH: launch_xz_arrow<3, MONTH>(s, lenient, f32, ag, tc, n, g, zhi, bin, xz, status, ctx->d_err); break;
      default: launch_xz_arrow<3, YEAR>(s, lenient, f32, ag, tc, n, g, zhi, bin, xz, status, ctx->d_err); break;
    }
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_xz2_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, int64_t n, int g, int lenient, int64_t* xz,
                           uint8_t* status, gm_batch_status* summary) {
  return xz_key_arrow(ctx, 2, geom, nullptr, n, g, WEEK, lenient, nullptr, xz, status, summary);
}

int gm_xz3_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, const gm_time_column* dtg, int64_t n, int g,
                           int period, int lenient, int16_t* bin, int64_t* xz, uint8_t* status,
                           gm_batch_status* summary) {
  return xz_key_arrow(ctx, 3, geom, dtg, n, g, period, lenient, bin, xz, status, summary);
}

int gm_arrow_points_to_columns(gm_ctx* ctx, const gm_geom_column* geom, int64_t n, double* x, double* y) {
  if (!ctx || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!point_col_ok(geom) || !x || !y) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  const ArrowPts g = to_pts(geom);
  if (geom->ordinal_bits == 32)
    hipLaunchKernelGGL((k_points_soa<true>), dim3(agrid(n)), dim3(ATPB), 0, ctx->stream, g, n, x, y);
  else
    hipLaunchKernelGGL((k_points_soa<false>), dim3(agrid(n)), dim3(ATPB), 0, ctx->stream, g, n, x, y);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

// The broadcast side of the join, from host Arrow vectors: de-interleave into the gm_polyset CSR
// (polygon -> parts -> rings -> vertices) and build the index as gm_pip_index_create_ex does.
int gm_pip_index_create_arrow(gm_ctx* ctx, const gm_geom_column* polys, int32_t n, int cells_per_poly,
                              gm_pip_index** out) {
  if (!ctx || !out || n < 0 || !polys) return GM_E_INVALID;
  if (polys->type != GM_GEOM_POLYGON && polys->type != GM_GEOM_MULTIPOLYGON) return GM_E_INVALID;
  if (n > 0 && !geom_col_ok(polys)) return GM_E_INVALID;
  const bool multi = polys->type == GM_GEOM_MULTIPOLYGON;
  std::vector<int32_t> ppo(1, 0), pro(1, 0), rvo(1, 0);
  std::vector<double> vx, vy;
  auto tuple = [&](int64_t j, double& x, double& y) {
    double o0, o1;
    if (polys->ordinal_bits == 32) {
      o0 = ((const float*)polys->coords)[2 * j]; o1 = ((const float*)polys->coords)[2 * j + 1];
    } else {
      o0 = ((const double*)polys->coords)[2 * j]; o1 = ((const double*)polys->coords)[2 * j + 1];
    }
    x = polys->flip_axis ? o0 : o1;
    y = polys->flip_axis ? o1 : o0;
  };
  auto add_polygon = [&](const int32_t* vert_off, int32_t r0, int32_t r1) {
    if (r1 <= r0) return;   // an empty polygon: no part
    for (int32_t r = r0; r < r1; ++r) {
      for (int32_t j = vert_off[r]; j < vert_off[r + 1]; ++j) {
        double x, y;
        tuple(j, x, y);
        vx.push_back(x);
        vy.push_back(y);
      }
      rvo.push_back((int32_t)vx.size());
    }
    pro.push_back((int32_t)rvo.size() - 1);
  };
  for (int32_t i = 0; i < n; ++i) {
    const int64_t b = polys->validity_offset + i;
    const bool valid = !polys->validity || ((polys->validity[b >> 3] >> (b & 7)) & 1u);
    if (valid) {
      if (multi) {
        for (int32_t p = polys->offsets[0][i]; p < polys->offsets[0][i + 1]; ++p)
          add_polygon(polys->offsets[2], polys->offsets[1][p], polys->offsets[1][p + 1]);
      } else {
        add_polygon(polys->offsets[1], polys->offsets[0][i], polys->offsets[0][i + 1]);
      }
    }
    ppo.push_back((int32_t)pro.size() - 1);
  }
  const gm_polyset ps{n, ppo.data(), pro.data(), rvo.data(), vx.data(), vy.data()};
  return gm_pip_index_create_ex(ctx, &ps, cells_per_poly, out);
}

}  // extern "C"
