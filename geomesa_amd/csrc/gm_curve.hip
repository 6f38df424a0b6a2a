// gm_curve.hip -- Z3/Z2 encode+decode, BinnedTime and XZ2/XZ3 envelope keys on gfx950.
//
// All of these are HBM-streaming element-wise kernels (34 B/point for the Z3 key, 32 B for the Z3
// invert, 24 B for Z2, 40/56 B for XZ): no reuse, no LDS, no MFMA.  Shape: 256-thread workgroups,
// each lane moves 2 consecutive elements with 16-byte loads/stores (one dwordx4 per column per
// lane), UNROLL independent pairs in flight per lane, fully coalesced per wave instruction
// (pair p of lane l in step u sits at block_base + u*256 + l).  One chunk per workgroup -- the
// grid is large (N / 2048 workgroups at UNROLL = 4), so all 256 CUs x 8 XCDs fill.
#include "gm_keys.hpp"

namespace gm {

#ifndef GM_CURVE_TPB
#define GM_CURVE_TPB 256
#endif
constexpr int TPB = GM_CURVE_TPB;
#ifndef GM_XZ_TPB
#define GM_XZ_TPB 128   // 64 / 128 / 256 / 512: profiles/r6/curve_block_unroll_ab.txt (128 and 64 ahead of 256 for both XZ kernels)
#endif
constexpr int XTPB = GM_XZ_TPB;   // the XZ kernels' block


// ------------------------------------------------------------------ Z3 key (epoch ms -> bin, z)

template <int PERIOD, bool LENIENT, bool STATUS, int UNROLL>
__global__ __launch_bounds__(TPB) void k_z3_index_key(const dv2* __restrict__ x, const dv2* __restrict__ y,
                                                      const lv2* __restrict__ t, int64_t n,
                                                      short2* __restrict__ bin, lv2* __restrict__ z,
                                                      uchar2* __restrict__ status, NDim lon, NDim lat, NDim tim,
                                                      int64_t* __restrict__ err) {
  // bins leave as one 16-B store per lane (the block's 2048 bins staged in LDS): 3.5% faster than a
  // 4-B store per pair (A/B on one box, round 2)
  __shared__ uint32_t s_bin[TPB * UNROLL];
  static_assert(UNROLL == 4, "staged bins: 4 pairs per lane");
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (TPB * UNROLL) + threadIdx.x;
  dv2 xv[UNROLL], yv[UNROLL];
  lv2 tv[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) {
      xv[u] = ld_stream(&x[p]);
      yv[u] = ld_stream(&y[p]);
      tv[u] = ld_stream(&t[p]);
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) {
      int16_t b0, b1;
      int64_t z0, z1;
      uint8_t s0 = z3_key_one<PERIOD, LENIENT>(xv[u].x, yv[u].x, tv[u].x, lon, lat, tim, b0, z0);
      uint8_t s1 = z3_key_one<PERIOD, LENIENT>(xv[u].y, yv[u].y, tv[u].y, lon, lat, tim, b1, z1);
      st_stream(lv2{z0, z1}, &z[p]);
      s_bin[u * TPB + threadIdx.x] = bin_pair(b0, b1);
      if (STATUS) status[p] = make_uchar2(s0, s1);
      if (s0) report_error(err, 2 * p, s0);
      if (s1) report_error(err, 2 * p + 1, s1);
    }
  }
  store_staged_bins<TPB>(s_bin, bin, npairs);
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    int16_t b;
    int64_t zz;
    uint8_t s = z3_key_one<PERIOD, LENIENT>(((const double*)x)[i], ((const double*)y)[i],
                                            ((const int64_t*)t)[i], lon, lat, tim, b, zz);
    ((int16_t*)bin)[i] = b;
    ((int64_t*)z)[i] = zz;
    if (STATUS) ((uint8_t*)status)[i] = s;
    if (s) report_error(err, i, s);
  }
}

// scalar fallback for unaligned columns
template <int PERIOD, bool LENIENT, bool STATUS>
__global__ __launch_bounds__(TPB) void k_z3_index_key_s(const double* __restrict__ x, const double* __restrict__ y,
                                                        const int64_t* __restrict__ t, int64_t n,
                                                        int16_t* __restrict__ bin, int64_t* __restrict__ z,
                                                        uint8_t* __restrict__ status, NDim lon, NDim lat, NDim tim,
                                                        int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int16_t b;
    int64_t zz;
    uint8_t s = z3_key_one<PERIOD, LENIENT>(x[i], y[i], t[i], lon, lat, tim, b, zz);
    bin[i] = b;
    z[i] = zz;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

// ------------------------------------------------------------------ Z3SFC.index (offset t)

template <bool LENIENT, bool STATUS>
__global__ __launch_bounds__(TPB) void k_z3_index(const double* __restrict__ x, const double* __restrict__ y,
                                                  const int64_t* __restrict__ t, int64_t n, int64_t* __restrict__ z,
                                                  uint8_t* __restrict__ status, NDim lon, NDim lat, NDim tim,
                                                  int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int64_t zz;
    uint8_t s = z3_index_one<LENIENT>(x[i], y[i], t[i], lon, lat, tim, zz);
    z[i] = zz;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

// ------------------------------------------------------------------ Z3SFC.invert

// plain 16-B stores as each pair is computed: 5.45-5.48 ms per 1B points against 5.51-5.63 for
// non-temporal ones and 5.42-5.58 with all of a lane's outputs computed before its stores, on one box
// (profiles/r6/invert_store_ab.txt); a second box ranked the store kinds the other way round within its
// noise (profiles/r6/store_kind_ab_box2.txt)
template <int UNROLL>
__global__ __launch_bounds__(TPB) void k_z3_invert(const lv2* __restrict__ z, int64_t n, dv2* __restrict__ x,
                                                   dv2* __restrict__ y, lv2* __restrict__ t, NDim lon,
                                                   NDim lat, NDim tim) {
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (TPB * UNROLL) + threadIdx.x;
  lv2 zv[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) zv[u] = ld_stream(&z[p]);
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) {
      const int64_t a = zv[u].x, b = zv[u].y;
      const dv2 xo{denormalize(lon, z3_combine(a)), denormalize(lon, z3_combine(b))};
      const dv2 yo{denormalize(lat, z3_combine(a >> 1)), denormalize(lat, z3_combine(b >> 1))};
      const lv2 to{jvm_d2l(denormalize(tim, z3_combine(a >> 2))), jvm_d2l(denormalize(tim, z3_combine(b >> 2)))};
      x[p] = xo; y[p] = yo; t[p] = to;
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    const int64_t a = ((const int64_t*)z)[i];
    ((double*)x)[i] = denormalize(lon, z3_combine(a));
    ((double*)y)[i] = denormalize(lat, z3_combine(a >> 1));
    ((int64_t*)t)[i] = jvm_d2l(denormalize(tim, z3_combine(a >> 2)));
  }
}

__global__ __launch_bounds__(TPB) void k_z3_invert_s(const int64_t* __restrict__ z, int64_t n, double* __restrict__ x,
                                                     double* __restrict__ y, int64_t* __restrict__ t, NDim lon,
                                                     NDim lat, NDim tim) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t a = z[i];
    x[i] = denormalize(lon, z3_combine(a));
    y[i] = denormalize(lat, z3_combine(a >> 1));
    t[i] = jvm_d2l(denormalize(tim, z3_combine(a >> 2)));
  }
}

// ------------------------------------------------------------------ Z2SFC.index / invert

template <bool LENIENT, bool STATUS, int UNROLL>
__global__ __launch_bounds__(TPB) void k_z2_index(const dv2* __restrict__ x, const dv2* __restrict__ y,
                                                  int64_t n, lv2* __restrict__ z, uchar2* __restrict__ status,
                                                  NDim lon, NDim lat, int64_t* __restrict__ err) {
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (TPB * UNROLL) + threadIdx.x;
  dv2 xv[UNROLL], yv[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) {
      xv[u] = ld_stream(&x[p]);
      yv[u] = ld_stream(&y[p]);
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) {
      int64_t z0, z1;
      uint8_t s0 = z2_index_one<LENIENT>(xv[u].x, yv[u].x, lon, lat, z0);
      uint8_t s1 = z2_index_one<LENIENT>(xv[u].y, yv[u].y, lon, lat, z1);
      st_stream(lv2{z0, z1}, &z[p]);
      if (STATUS) status[p] = make_uchar2(s0, s1);
      if (s0) report_error(err, 2 * p, s0);
      if (s1) report_error(err, 2 * p + 1, s1);
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    int64_t zz;
    uint8_t s = z2_index_one<LENIENT>(((const double*)x)[i], ((const double*)y)[i], lon, lat, zz);
    ((int64_t*)z)[i] = zz;
    if (STATUS) ((uint8_t*)status)[i] = s;
    if (s) report_error(err, i, s);
  }
}

template <bool LENIENT, bool STATUS>
__global__ __launch_bounds__(TPB) void k_z2_index_s(const double* __restrict__ x, const double* __restrict__ y,
                                                    int64_t n, int64_t* __restrict__ z, uint8_t* __restrict__ status,
                                                    NDim lon, NDim lat, int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int64_t zz;
    uint8_t s = z2_index_one<LENIENT>(x[i], y[i], lon, lat, zz);
    z[i] = zz;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

template <int UNROLL>
__global__ __launch_bounds__(TPB) void k_z2_invert(const lv2* __restrict__ z, int64_t n, dv2* __restrict__ x,
                                                   dv2* __restrict__ y, NDim lon, NDim lat) {
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (TPB * UNROLL) + threadIdx.x;
  lv2 zv[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) zv[u] = ld_stream(&z[p]);
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * TPB;
    if (p < npairs) {
      const int64_t a = zv[u].x, b = zv[u].y;
      st_stream(dv2{denormalize(lon, z2_combine(a)), denormalize(lon, z2_combine(b))},
                                  &x[p]);
      st_stream(
          dv2{denormalize(lat, z2_combine(a >> 1)), denormalize(lat, z2_combine(b >> 1))}, &y[p]);
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    const int64_t a = ((const int64_t*)z)[i];
    ((double*)x)[i] = denormalize(lon, z2_combine(a));
    ((double*)y)[i] = denormalize(lat, z2_combine(a >> 1));
  }
}

__global__ __launch_bounds__(TPB) void k_z2_invert_s(const int64_t* __restrict__ z, int64_t n, double* __restrict__ x,
                                                     double* __restrict__ y, NDim lon, NDim lat) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    const int64_t a = z[i];
    x[i] = denormalize(lon, z2_combine(a));
    y[i] = denormalize(lat, z2_combine(a >> 1));
  }
}

// ------------------------------------------------------------------ BinnedTime

template <int PERIOD, bool STATUS>
__global__ __launch_bounds__(TPB) void k_binned_time(const int64_t* __restrict__ t, int64_t n,
                                                     int16_t* __restrict__ bin, int64_t* __restrict__ off,
                                                     uint8_t* __restrict__ status, int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int16_t b;
    int64_t o;
    uint8_t s = binned_time<PERIOD>(t[i], b, o);
    bin[i] = b;
    off[i] = o;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

template <bool LENIENT, bool STATUS>
__global__ __launch_bounds__(TPB) void k_xz2_index(const double* __restrict__ xmin, const double* __restrict__ ymin,
                                                   const double* __restrict__ xmax, const double* __restrict__ ymax,
                                                   int64_t n, int g, int64_t* __restrict__ out,
                                                   uint8_t* __restrict__ status, int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int64_t o;
    uint8_t s = xz2_one<LENIENT>(g, xmin[i], ymin[i], xmax[i], ymax[i], o);
    out[i] = o;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

template <bool LENIENT, bool STATUS>
__global__ __launch_bounds__(TPB) void k_xz3_index(const double* __restrict__ xmin, const double* __restrict__ ymin,
                                                   const double* __restrict__ zmin, const double* __restrict__ xmax,
                                                   const double* __restrict__ ymax, const double* __restrict__ zmax,
                                                   int64_t n, int g, double zhi, int64_t* __restrict__ out,
                                                   uint8_t* __restrict__ status, int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int64_t o;
    uint8_t s = xz3_one<LENIENT>(g, zhi, xmin[i], ymin[i], zmin[i], xmax[i], ymax[i], zmax[i], o);
    out[i] = o;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

// XZ3IndexKeySpace.toIndexKey (idx/index/z3/XZ3IndexKeySpace.scala:60-95) over envelope + dtg columns:
// BinnedTime(dtg) (null dtg column -> 0) outside the lenient try, then XZ3SFC.index of the envelope at
// the period offset.  A failed row gets bin 0 and key 0 and its status.
template <int PERIOD, bool LENIENT, bool STATUS>
__global__ __launch_bounds__(TPB) void k_xz3_index_key(const double* __restrict__ xmin, const double* __restrict__ ymin,
                                                       const double* __restrict__ xmax, const double* __restrict__ ymax,
                                                       const int64_t* __restrict__ t_ms, int64_t n, int g, double zhi,
                                                       int16_t* __restrict__ bin, int64_t* __restrict__ out,
                                                       uint8_t* __restrict__ status, int64_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * TPB) {
    int64_t o = 0, off = 0;
    int16_t b = 0;
    uint8_t s = binned_time<PERIOD>(t_ms ? t_ms[i] : 0, b, off);
    if (s == ST_OK) {
      const double t = (double)off;
      s = xz3_one<LENIENT>(g, zhi, xmin[i], ymin[i], t, xmax[i], ymax[i], t, o);
    }
    if (s != ST_OK) { o = 0; b = 0; }
    out[i] = o;
    bin[i] = b;
    if (STATUS) status[i] = s;
    if (s) report_error(err, i, s);
  }
}

// 16-B form: 2 envelopes per lane per column (one dwordx4 each), UNROLL pairs in flight per lane,
// the same coalesced layout as the Z3 key kernel; the odd last envelope goes to lane 0 of block 0.
template <bool LENIENT, bool STATUS, int UNROLL>
__global__ __launch_bounds__(XTPB) void k_xz2_index_v(const dv2* __restrict__ xmin, const dv2* __restrict__ ymin,
                                                     const dv2* __restrict__ xmax, const dv2* __restrict__ ymax,
                                                     int64_t n, int g, lv2* __restrict__ out,
                                                     uchar2* __restrict__ status, int64_t* __restrict__ err) {
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (XTPB * UNROLL) + threadIdx.x;
  dv2 a[UNROLL], b[UNROLL], c[UNROLL], d[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * XTPB;
    if (p < npairs) {
      a[u] = ld_stream(&xmin[p]); b[u] = ld_stream(&ymin[p]);
      c[u] = ld_stream(&xmax[p]); d[u] = ld_stream(&ymax[p]);
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * XTPB;
    if (p < npairs) {
      int64_t o0, o1;
      const uint8_t s0 = xz2_one<LENIENT>(g, a[u].x, b[u].x, c[u].x, d[u].x, o0);
      const uint8_t s1 = xz2_one<LENIENT>(g, a[u].y, b[u].y, c[u].y, d[u].y, o1);
      st_stream(lv2{o0, o1}, &out[p]);
      if (STATUS) status[p] = make_uchar2(s0, s1);
      if (s0) report_error(err, 2 * p, s0);
      if (s1) report_error(err, 2 * p + 1, s1);
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    int64_t o;
    const uint8_t s = xz2_one<LENIENT>(g, ((const double*)xmin)[i], ((const double*)ymin)[i],
                                       ((const double*)xmax)[i], ((const double*)ymax)[i], o);
    ((int64_t*)out)[i] = o;
    if (STATUS) ((uint8_t*)status)[i] = s;
    if (s) report_error(err, i, s);
  }
}

template <bool LENIENT, bool STATUS, int UNROLL>
__global__ __launch_bounds__(XTPB) void k_xz3_index_v(const dv2* __restrict__ xmin, const dv2* __restrict__ ymin,
                                                     const dv2* __restrict__ zmin, const dv2* __restrict__ xmax,
                                                     const dv2* __restrict__ ymax, const dv2* __restrict__ zmax,
                                                     int64_t n, int g, double zhi, lv2* __restrict__ out,
                                                     uchar2* __restrict__ status, int64_t* __restrict__ err) {
  const int64_t npairs = n >> 1;
  const int64_t base = (int64_t)blockIdx.x * (XTPB * UNROLL) + threadIdx.x;
  dv2 a[UNROLL], b[UNROLL], c[UNROLL], d[UNROLL], e[UNROLL], f[UNROLL];
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * XTPB;
    if (p < npairs) {
      a[u] = ld_stream(&xmin[p]); b[u] = ld_stream(&ymin[p]); c[u] = ld_stream(&zmin[p]);
      d[u] = ld_stream(&xmax[p]); e[u] = ld_stream(&ymax[p]); f[u] = ld_stream(&zmax[p]);
    }
  }
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t p = base + (int64_t)u * XTPB;
    if (p < npairs) {
      int64_t o0, o1;
      const uint8_t s0 = xz3_one<LENIENT>(g, zhi, a[u].x, b[u].x, c[u].x, d[u].x, e[u].x, f[u].x, o0);
      const uint8_t s1 = xz3_one<LENIENT>(g, zhi, a[u].y, b[u].y, c[u].y, d[u].y, e[u].y, f[u].y, o1);
      st_stream(lv2{o0, o1}, &out[p]);
      if (STATUS) status[p] = make_uchar2(s0, s1);
      if (s0) report_error(err, 2 * p, s0);
      if (s1) report_error(err, 2 * p + 1, s1);
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t i = n - 1;
    int64_t o;
    const uint8_t s = xz3_one<LENIENT>(g, zhi, ((const double*)xmin)[i], ((const double*)ymin)[i],
                                       ((const double*)zmin)[i], ((const double*)xmax)[i], ((const double*)ymax)[i],
                                       ((const double*)zmax)[i], o);
    ((int64_t*)out)[i] = o;
    if (STATUS) ((uint8_t*)status)[i] = s;
    if (s) report_error(err, i, s);
  }
}

// ------------------------------------------------------------------ host-side launchers

// pairs per lane; tuning sweeps build variants with -DGM_UNROLL_INV=... (tools/jx_build.sh, tools/curve_ab.sh).
// The key kernel's LDS bin staging fixes UNROLL_KEY at 4; XZ 1 / 2 / 4 were within noise.
#ifndef GM_UNROLL_KEY
#define GM_UNROLL_KEY 4
#endif
#ifndef GM_UNROLL_INV
#define GM_UNROLL_INV 2   // 1 / 2 / 4 / 8: profiles/r2_curve_unroll_sweep.txt (2 beat 4 in every same-box pair)
#endif
#ifndef GM_UNROLL_XZ
#define GM_UNROLL_XZ 2
#endif
constexpr int UNROLL_KEY = GM_UNROLL_KEY;
constexpr int UNROLL_INV = GM_UNROLL_INV;
#ifndef GM_UNROLL_INV2
#define GM_UNROLL_INV2 1   // the Z2 inverse: 1 pair per lane 3.68-3.83 vs 2 pairs 4.12-4.23 ms (profiles/r6/invert_unroll_ab.txt)
#endif
constexpr int UNROLL_INV2 = GM_UNROLL_INV2;
constexpr int UNROLL_XZ = GM_UNROLL_XZ;
#ifndef GM_UNROLL_Z2
#define GM_UNROLL_Z2 1   // round 6: 1 pair per lane 3.635-3.640 vs 2 pairs 3.84-4.01 ms per 1B points (profiles/r6/curve_block_unroll_ab.txt); round 2: 2 / 4 / 8 3.91 / 3.94-3.98 / 4.09-4.11
#endif
constexpr int UNROLL_Z2 = GM_UNROLL_Z2;

inline unsigned stride_grid(int64_t n) {
  int64_t b = (n + TPB - 1) / TPB;
  if (b > 256 * 16) b = 256 * 16;
  return (unsigned)(b < 1 ? 1 : b);
}

template <int PERIOD, bool LENIENT, bool STATUS>
void launch_key(hipStream_t s, const double* x, const double* y, const int64_t* t, int64_t n, int16_t* bin,
                int64_t* z, uint8_t* status, NDim lon, NDim lat, NDim tim, int64_t* err, bool vec) {
  if (vec) {
    unsigned grid = grid_for((n >> 1) > 0 ? (n >> 1) : 1, (int64_t)TPB * UNROLL_KEY);
    hipLaunchKernelGGL((k_z3_index_key<PERIOD, LENIENT, STATUS, UNROLL_KEY>), dim3(grid), dim3(TPB), 0, s,
                       (const dv2*)x, (const dv2*)y, (const lv2*)t, n, (short2*)bin, (lv2*)z,
                       (uchar2*)status, lon, lat, tim, err);
  } else {
    hipLaunchKernelGGL((k_z3_index_key_s<PERIOD, LENIENT, STATUS>), dim3(stride_grid(n)), dim3(TPB), 0, s, x, y, t,
                       n, bin, z, status, lon, lat, tim, err);
  }
}

template <int PERIOD>
void launch_key_p(hipStream_t s, const double* x, const double* y, const int64_t* t, int64_t n, int16_t* bin,
                  int64_t* z, uint8_t* status, NDim lon, NDim lat, NDim tim, int64_t* err, bool lenient, bool vec) {
  if (lenient) {
    if (status) launch_key<PERIOD, true, true>(s, x, y, t, n, bin, z, status, lon, lat, tim, err, vec);
    else launch_key<PERIOD, true, false>(s, x, y, t, n, bin, z, status, lon, lat, tim, err, vec);
  } else {
    if (status) launch_key<PERIOD, false, true>(s, x, y, t, n, bin, z, status, lon, lat, tim, err, vec);
    else launch_key<PERIOD, false, false>(s, x, y, t, n, bin, z, status, lon, lat, tim, err, vec);
  }
}


}  // namespace gm

using namespace gm;

extern "C" {

int gm_z3_index_key(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n, int period,
                    int lenient, int16_t* bin, int64_t* z, uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || !valid_period(period)) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!x || !y || !t_ms || !bin || !z) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const NDim lon = lon_dim(21), lat = lat_dim(21), tim = time_dim(period, 21);
  const bool vec = aligned16(x) && aligned16(y) && aligned16(t_ms) && aligned16(z) &&
                   (((uintptr_t)bin & 3u) == 0) && (((uintptr_t)status & 1u) == 0);
  switch (period) {
    case DAY: launch_key_p<DAY>(ctx->stream, x, y, t_ms, n, bin, z, status, lon, lat, tim, ctx->d_err, lenient, vec); break;
    case WEEK: launch_key_p<WEEK>(ctx->stream, x, y, t_ms, n, bin, z, status, lon, lat, tim, ctx->d_err, lenient, vec); break;
    case MONTH: launch_key_p<MONTH>(ctx->stream, x, y, t_ms, n, bin, z, status, lon, lat, tim, ctx->d_err, lenient, vec); break;
    default: launch_key_p<YEAR>(ctx->stream, x, y, t_ms, n, bin, z, status, lon, lat, tim, ctx->d_err, lenient, vec); break;
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_z3_index(gm_ctx* ctx, const double* x, const double* y, const int64_t* t, int64_t n, int period,
                int precision, int lenient, int64_t* z, uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || !valid_period(period) || precision < 1 || precision > 21) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!x || !y || !t || !z) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const NDim lon = lon_dim(precision), lat = lat_dim(precision), tim = time_dim(period, precision);
  const unsigned grid = stride_grid(n);
  if (lenient) {
    if (status) hipLaunchKernelGGL((k_z3_index<true, true>), dim3(grid), dim3(TPB), 0, ctx->stream, x, y, t, n, z, status, lon, lat, tim, ctx->d_err);
    else hipLaunchKernelGGL((k_z3_index<true, false>), dim3(grid), dim3(TPB), 0, ctx->stream, x, y, t, n, z, status, lon, lat, tim, ctx->d_err);
  } else {
    if (status) hipLaunchKernelGGL((k_z3_index<false, true>), dim3(grid), dim3(TPB), 0, ctx->stream, x, y, t, n, z, status, lon, lat, tim, ctx->d_err);
    else hipLaunchKernelGGL((k_z3_index<false, false>), dim3(grid), dim3(TPB), 0, ctx->stream, x, y, t, n, z, status, lon, lat, tim, ctx->d_err);
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_z3_invert(gm_ctx* ctx, const int64_t* z, int64_t n, int period, int precision, double* x, double* y,
                 int64_t* t) {
  if (!ctx || n < 0 || !valid_period(period) || precision < 1 || precision > 21) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!z || !x || !y || !t) return GM_E_INVALID;
  const NDim lon = lon_dim(precision), lat = lat_dim(precision), tim = time_dim(period, precision);
  if (aligned16(z) && aligned16(x) && aligned16(y) && aligned16(t)) {
    unsigned grid = grid_for((n >> 1) > 0 ? (n >> 1) : 1, (int64_t)TPB * UNROLL_INV);
    hipLaunchKernelGGL((k_z3_invert<UNROLL_INV>), dim3(grid), dim3(TPB), 0, ctx->stream, (const lv2*)z, n,
                       (dv2*)x, (dv2*)y, (lv2*)t, lon, lat, tim);
  } else {
    hipLaunchKernelGGL(k_z3_invert_s, dim3(stride_grid(n)), dim3(TPB), 0, ctx->stream, z, n, x, y, t, lon, lat, tim);
  }
  GM_CHECK_LAUNCH();
  return GM_OK;
}

int gm_z2_index(gm_ctx* ctx, const double* x, const double* y, int64_t n, int precision, int lenient, int64_t* z,
                uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || precision < 1 || precision > 31) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!x || !y || !z) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const NDim lon = lon_dim(precision), lat = lat_dim(precision);
  const bool vec = aligned16(x) && aligned16(y) && aligned16(z) && (((uintptr_t)status & 1u) == 0);
  hipStream_t s = ctx->stream;
  if (vec) {
    unsigned grid = grid_for((n >> 1) > 0 ? (n >> 1) : 1, (int64_t)TPB * UNROLL_Z2);
    const dv2* x2 = (const dv2*)x; const dv2* y2 = (const dv2*)y;
    lv2* z2 = (lv2*)z; uchar2* s2 = (uchar2*)status;
    if (lenient) {
      if (status) hipLaunchKernelGGL((k_z2_index<true, true, UNROLL_Z2>), dim3(grid), dim3(TPB), 0, s, x2, y2, n, z2, s2, lon, lat, ctx->d_err);
      else hipLaunchKernelGGL((k_z2_index<true, false, UNROLL_Z2>), dim3(grid), dim3(TPB), 0, s, x2, y2, n, z2, s2, lon, lat, ctx->d_err);
    } else {
      if (status) hipLaunchKernelGGL((k_z2_index<false, true, UNROLL_Z2>), dim3(grid), dim3(TPB), 0, s, x2, y2, n, z2, s2, lon, lat, ctx->d_err);
      else hipLaunchKernelGGL((k_z2_index<false, false, UNROLL_Z2>), dim3(grid), dim3(TPB), 0, s, x2, y2, n, z2, s2, lon, lat, ctx->d_err);
    }
  } else {
    unsigned grid = stride_grid(n);
    if (lenient) {
      if (status) hipLaunchKernelGGL((k_z2_index_s<true, true>), dim3(grid), dim3(TPB), 0, s, x, y, n, z, status, lon, lat, ctx->d_err);
      else hipLaunchKernelGGL((k_z2_index_s<true, false>), dim3(grid), dim3(TPB), 0, s, x, y, n, z, status, lon, lat, ctx->d_err);
    } else {
      if (status) hipLaunchKernelGGL((k_z2_index_s<false, true>), dim3(grid), dim3(TPB), 0, s, x, y, n, z, status, lon, lat, ctx->d_err);
      else hipLaunchKernelGGL((k_z2_index_s<false, false>), dim3(grid), dim3(TPB), 0, s, x, y, n, z, status, lon, lat, ctx->d_err);
    }
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_z2_invert(gm_ctx* ctx, const int64_t* z, int64_t n, int precision, double* x, double* y) {
  if (!ctx || n < 0 || precision < 1 || precision > 31) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!z || !x || !y) return GM_E_INVALID;
  const NDim lon = lon_dim(precision), lat = lat_dim(precision);
  if (aligned16(z) && aligned16(x) && aligned16(y)) {
    unsigned grid = grid_for((n >> 1) > 0 ? (n >> 1) : 1, (int64_t)TPB * UNROLL_INV2);
    hipLaunchKernelGGL((k_z2_invert<UNROLL_INV2>), dim3(grid), dim3(TPB), 0, ctx->stream, (const lv2*)z, n,
                       (dv2*)x, (dv2*)y, lon, lat);
  } else {
    hipLaunchKernelGGL(k_z2_invert_s, dim3(stride_grid(n)), dim3(TPB), 0, ctx->stream, z, n, x, y, lon, lat);
  }
  GM_CHECK_LAUNCH();
  return GM_OK;
}

int gm_binned_time(gm_ctx* ctx, const int64_t* t_ms, int64_t n, int period, int16_t* bin, int64_t* offset,
                   uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || !valid_period(period)) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!t_ms || !bin || !offset) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const unsigned grid = stride_grid(n);
  hipStream_t s = ctx->stream;
#define GM_BT(P)                                                                                          \
  if (status) hipLaunchKernelGGL((k_binned_time<P, true>), dim3(grid), dim3(TPB), 0, s, t_ms, n, bin, offset, status, ctx->d_err); \
  else hipLaunchKernelGGL((k_binned_time<P, false>), dim3(grid), dim3(TPB), 0, s, t_ms, n, bin, offset, status, ctx->d_err);
  switch (period) {
    case DAY: GM_BT(DAY) break;
    case WEEK: GM_BT(WEEK) break;
    case MONTH: GM_BT(MONTH) break;
    default: GM_BT(YEAR) break;
  }
#undef GM_BT
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_xz2_index(gm_ctx* ctx, const double* xmin, const double* ymin, const double* xmax, const double* ymax,
                 int64_t n, int g, int lenient, int64_t* out, uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || g < 1 || g > 30) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!xmin || !ymin || !xmax || !ymax || !out) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const unsigned grid = stride_grid(n);
  hipStream_t s = ctx->stream;
  if (aligned16(xmin) && aligned16(ymin) && aligned16(xmax) && aligned16(ymax) && aligned16(out) &&
      (((uintptr_t)status & 1u) == 0)) {
    const unsigned vg = grid_for((n >> 1) > 0 ? (n >> 1) : 1, (int64_t)XTPB * UNROLL_XZ);
    const dv2 *a = (const dv2*)xmin, *b = (const dv2*)ymin, *c = (const dv2*)xmax, *d = (const dv2*)ymax;
    lv2* o = (lv2*)out;
    uchar2* st = (uchar2*)status;
    if (lenient) {
      if (status) hipLaunchKernelGGL((k_xz2_index_v<true, true, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, n, g, o, st, ctx->d_err);
      else hipLaunchKernelGGL((k_xz2_index_v<true, false, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, n, g, o, st, ctx->d_err);
    } else {
      if (status) hipLaunchKernelGGL((k_xz2_index_v<false, true, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, n, g, o, st, ctx->d_err);
      else hipLaunchKernelGGL((k_xz2_index_v<false, false, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, n, g, o, st, ctx->d_err);
    }
  } else if (lenient) {
    if (status) hipLaunchKernelGGL((k_xz2_index<true, true>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, xmax, ymax, n, g, out, status, ctx->d_err);
    else hipLaunchKernelGGL((k_xz2_index<true, false>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, xmax, ymax, n, g, out, status, ctx->d_err);
  } else {
    if (status) hipLaunchKernelGGL((k_xz2_index<false, true>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, xmax, ymax, n, g, out, status, ctx->d_err);
    else hipLaunchKernelGGL((k_xz2_index<false, false>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, xmax, ymax, n, g, out, status, ctx->d_err);
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_xz3_index(gm_ctx* ctx, const double* xmin, const double* ymin, const double* zmin, const double* xmax,
                 const double* ymax, const double* zmax, int64_t n, int g, int period, int lenient, int64_t* out,
                 uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || g < 1 || g > 20 || !valid_period(period)) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!xmin || !ymin || !zmin || !xmax || !ymax || !zmax || !out) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const unsigned grid = stride_grid(n);
  const double zhi = (double)max_offset(period);
  hipStream_t s = ctx->stream;
  if (aligned16(xmin) && aligned16(ymin) && aligned16(zmin) && aligned16(xmax) && aligned16(ymax) &&
      aligned16(zmax) && aligned16(out) && (((uintptr_t)status & 1u) == 0)) {
    const unsigned vg = grid_for((n >> 1) > 0 ? (n >> 1) : 1, (int64_t)XTPB * UNROLL_XZ);
    const dv2 *a = (const dv2*)xmin, *b = (const dv2*)ymin, *c = (const dv2*)zmin;
    const dv2 *d = (const dv2*)xmax, *e = (const dv2*)ymax, *f = (const dv2*)zmax;
    lv2* o = (lv2*)out;
    uchar2* st = (uchar2*)status;
    if (lenient) {
      if (status) hipLaunchKernelGGL((k_xz3_index_v<true, true, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, e, f, n, g, zhi, o, st, ctx->d_err);
      else hipLaunchKernelGGL((k_xz3_index_v<true, false, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, e, f, n, g, zhi, o, st, ctx->d_err);
    } else {
      if (status) hipLaunchKernelGGL((k_xz3_index_v<false, true, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, e, f, n, g, zhi, o, st, ctx->d_err);
      else hipLaunchKernelGGL((k_xz3_index_v<false, false, UNROLL_XZ>), dim3(vg), dim3(XTPB), 0, s, a, b, c, d, e, f, n, g, zhi, o, st, ctx->d_err);
    }
  } else if (lenient) {
    if (status) hipLaunchKernelGGL((k_xz3_index<true, true>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, zmin, xmax, ymax, zmax, n, g, zhi, out, status, ctx->d_err);
    else hipLaunchKernelGGL((k_xz3_index<true, false>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, zmin, xmax, ymax, zmax, n, g, zhi, out, status, ctx->d_err);
  } else {
    if (status) hipLaunchKernelGGL((k_xz3_index<false, true>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, zmin, xmax, ymax, zmax, n, g, zhi, out, status, ctx->d_err);
    else hipLaunchKernelGGL((k_xz3_index<false, false>), dim3(grid), dim3(TPB), 0, s, xmin, ymin, zmin, xmax, ymax, zmax, n, g, zhi, out, status, ctx->d_err);
  }
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

int gm_xz3_index_key(gm_ctx* ctx, const double* xmin, const double* ymin, const double* xmax, const double* ymax,
                     const int64_t* t_ms, int64_t n, int g, int period, int lenient, int16_t* bin, int64_t* xz,
                     uint8_t* status, gm_batch_status* summary) {
  if (!ctx || n < 0 || g < 1 || g > 20 || !valid_period(period)) return GM_E_INVALID;
  if (n == 0) { if (summary) *summary = gm_batch_status{0, -1, 0, 0}; return GM_OK; }
  if (!xmin || !ymin || !xmax || !ymax || !bin || !xz) return GM_E_INVALID;
  int rc = begin_summary(ctx, summary);
  if (rc) return rc;
  const unsigned grid = stride_grid(n);
  const double zhi = (double)max_offset(period);
  hipStream_t s = ctx->stream;
#define GM_XZ3K(P)                                                                                                   \
  do {                                                                                                               \
    auto k = lenient ? (status ? k_xz3_index_key<P, true, true> : k_xz3_index_key<P, true, false>)                  \
                     : (status ? k_xz3_index_key<P, false, true> : k_xz3_index_key<P, false, false>);               \
    hipLaunchKernelGGL(k, dim3(grid), dim3(TPB), 0, s, xmin, ymin, xmax, ymax, t_ms, n, g, zhi, bin, xz, status,     \
                       ctx->d_err);                                                                                  \
  } while (0)
  switch (period) {
    case GM_DAY: GM_XZ3K(GM_DAY); break;
    case GM_WEEK: GM_XZ3K(GM_WEEK); break;
    case GM_MONTH: GM_XZ3K(GM_MONTH); break;
    default: GM_XZ3K(GM_YEAR); break;
  }
#undef GM_XZ3K
  GM_CHECK_LAUNCH();
  return end_summary(ctx, summary);
}

}  // extern "C"
