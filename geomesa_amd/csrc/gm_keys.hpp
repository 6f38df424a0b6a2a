// gm_keys.hpp -- per-element key bodies (Z3 / Z2 / XZ2 / XZ3 index with the JVM's bounds checks)
// and the streaming load/store helpers, shared by the column kernels (gm_curve.hip) and the Arrow
// kernels (gm_arrow.hip).
#pragma once

#include "gm_internal.hpp"

namespace gm {

// every column kernel streams: non-temporal loads and stores (the data is touched once).
// Loads under a per-lane branch (`if (p < n) v = load(p)`) cannot be counted by the compiler: it
// waits for every outstanding load (s_waitcnt vmcnt(0)) at the branch's end, and a select around a
// load (`v = p < n ? load(p) : 0`) is waited for before the next load is even issued.  Where a
// batch of loads must be in flight together (the sort passes, the histogram's prefetch) it is issued
// unconditionally, past-the-end lanes reading the last valid element (index clamped, result unused).
// The per-pair kernels keep their conditional batches (all of a lane's loads are issued before the
// one wait anyway): the unconditional form, which lets each pair's arithmetic start on its own loads,
// measured 1-3% slower for the Z3 key and no faster for XZ and the fused filter
// (profiles/r5/unconditional_loads_ab.txt, unconditional_loads_xz_query_ab.txt).
template <class T>
__device__ __forceinline__ T ld_stream(const T* p) {
  return __builtin_nontemporal_load(p);
}
template <class T>
__device__ __forceinline__ void st_stream(T v, T* p) {
  __builtin_nontemporal_store(v, p);
}

// Bins of a key kernel's block leave as one 16-B store per lane: pair j of the block (pairs
// [block * TPB * 4, +TPB * 4)) sits at s_bin[j] as bin0 | bin1 << 16, and lane l stores pairs
// 4l .. 4l + 3 (a 4-B store per pair otherwise; bin columns are only 4-B aligned).  Every thread of
// the block calls it (one barrier).
template <int TPB>
__device__ __forceinline__ void store_staged_bins(const uint32_t* s_bin, short2* __restrict__ bin, int64_t npairs) {
  typedef unsigned int uv4 __attribute__((ext_vector_type(4)));
  __syncthreads();
  const int64_t q = (int64_t)blockIdx.x * (TPB * 4) + 4 * (int64_t)threadIdx.x;
  if (q + 3 < npairs && ((uintptr_t)bin & 15u) == 0) {
    __builtin_nontemporal_store(*(const uv4*)&s_bin[4 * threadIdx.x], (uv4*)&bin[q]);
  } else {
    for (int k = 0; k < 4; ++k)
      if (q + k < npairs) ((uint32_t*)bin)[q + k] = s_bin[4 * threadIdx.x + k];
  }
}

__device__ __forceinline__ uint32_t bin_pair(int16_t b0, int16_t b1) {
  return (uint32_t)(uint16_t)b0 | ((uint32_t)(uint16_t)b1 << 16);
}

// ------------------------------------------------------------------ per-element bodies

// Z3SFC.index (z3/curve/Z3SFC.scala:37-52); t is the offset within the period (Long)
template <bool LENIENT>
__device__ __forceinline__ uint8_t z3_index_one(double x, double y, int64_t t, const NDim& lon, const NDim& lat,
                                                const NDim& tim, int64_t& z) {
  double td = (double)t;  // Long compared to / normalized as Double
  bool inb = x >= lon.min && x <= lon.max && y >= lat.min && y <= lat.max && td >= tim.min && td <= tim.max;
  if (!inb) {
    if (!LENIENT) { z = 0; return ST_OUT_OF_BOUNDS; }
    // lenientIndex (Z3SFC.scala:47-52): NaN falls through every comparison
    x = x < lon.min ? lon.min : (x > lon.max ? lon.max : x);
    y = y < lat.min ? lat.min : (y > lat.max ? lat.max : y);
    td = td < tim.min ? tim.min : (td > tim.max ? tim.max : td);
  }
  z = z3_apply(normalize(lon, x), normalize(lat, y), normalize(tim, td));
  return ST_OK;
}

// Z3IndexKeySpace.toIndexKey (idx/index/z3/Z3IndexKeySpace.scala:71-76): BinnedTime throws even
// when lenient (it sits outside the try at :74); then sfc.index(x, y, offset, lenient)
template <int PERIOD, bool LENIENT>
__device__ __forceinline__ uint8_t z3_key_one(double x, double y, int64_t ms, const NDim& lon, const NDim& lat,
                                              const NDim& tim, int16_t& bin, int64_t& z) {
  int64_t off;
  uint8_t st = binned_time<PERIOD>(ms, bin, off);
  if (st == ST_OK) st = z3_index_one<LENIENT>(x, y, off, lon, lat, tim, z);
  if (st != ST_OK) { bin = 0; z = 0; }
  return st;
}

// Z3.split through an LDS table of spread3_11 (2048 entries): two lookups per dimension replace the
// two 8-op magic-number spreads (the Z3Histogram kernels, gm_stats.hip)
__device__ __forceinline__ uint64_t z3_split_tab(int32_t value, const uint32_t* sp) {
  const uint32_t v = (uint32_t)value & 0x1fffffu;
  return ((uint64_t)sp[v >> 11] << 33) | (uint64_t)sp[v & 0x7ffu];
}
__device__ __forceinline__ void fill_spread_table(uint32_t* sp, int tid, int nthreads) {
  for (int i = tid; i < 2048; i += nthreads) sp[i] = spread3_11((uint32_t)i);
}
template <bool LENIENT>
__device__ __forceinline__ uint8_t z2_index_one(double x, double y, const NDim& lon, const NDim& lat,
                                                int64_t& z) {
  bool inb = x >= lon.min && x <= lon.max && y >= lat.min && y <= lat.max;
  if (!inb) {
    if (!LENIENT) { z = 0; return ST_OUT_OF_BOUNDS; }
    x = x < lon.min ? lon.min : (x > lon.max ? lon.max : x);
    y = y < lat.min ? lat.min : (y > lat.max ? lat.max : y);
  }
  z = z2_apply(normalize(lon, x), normalize(lat, y));
  return ST_OK;
}

// ------------------------------------------------------------------ XZ2 / XZ3

__device__ __forceinline__ double jmax(double a, double b) { return a >= b ? a : b; }  // operands never NaN/-0 here

// The XZ sequence code without the per-level FP loop.  XZ2SFC.sequenceCode (XZ2SFC.scala:264-286)
// halves [x0, x1] `length` times and compares the normalized minimum with the exact dyadic centre:
// at level i the cell is [k 2^-i, (k + 1) 2^-i) and `v < centre` is bit i+1 of v's binary
// expansion, so the `length` answers are the leading bits of floor(v 2^length) (v = 1.0 takes the
// upper half every time: 2^length - 1).  With q_i = x_i + 2 y_i (+ 4 z_i) the code is
//   cs = sum_{i<L} (1 + q_i (B^(g-i) - 1) / (B - 1)),  B = 4 (8)
//      = L + (interleave(x, y[, z]) B^(g-L+1) - sum_i q_i) / (B - 1),
// the interleave being exactly the Z2 / Z3 bit spread.  Integer-only and exact.
__device__ __forceinline__ uint32_t xz_cell(double v, int L) {
  const double s = floor(__dmul_rn(v, ldexp(1.0, L)));   // exact: power-of-two scaling
  const uint32_t m = (1u << L) - 1u;                      // L <= 30
  const uint32_t c = (uint32_t)s;                         // v in [0, 1] -> s in [0, 2^L]
  return c > m ? m : c;
}

// the `length` predicate (XZ2SFC.scala:66-74): mx <= floor(mn / w2) * w2 + 2 * w2 with w2 = 2^-(l1+1).
// Dividing by a power of two is exact, so mn * 2^(l1+1) gives the identical double.
__device__ __forceinline__ bool xz_fits(double mn, double mx, double w2, double inv_w2) {
  return mx <= __dadd_rn(__dmul_rn(floor(__dmul_rn(mn, inv_w2)), w2), __dmul_rn(2.0, w2));
}

// RN(a / b) for the constant spans b = 360, 180 and a = v - lo in {0} u [2^-45, b] (v a finite clamped
// coordinate, so a is 0 or at least ulp(180)): y = RN(1 / b) has y b = 1 + 0.34 * 2^-53 for both spans, so
// q = RN(a y) is within one ulp of a / b, r = a - q b is exact in one fma, and RN(q + r y) is the
// correctly rounded quotient (Markstein's correction theorem; no underflow on this domain).  Three f64
// ops against the ~10 of the IEEE divide sequence; checked against a / b on the host (tools/div_check.c:
// random, every exponent down to 2^-45, +-3 ulp around every j b / 2^20) and bit-compared with the
// oracle by the GPU parity tests.
__device__ __forceinline__ double div_span(double a, double b, double y) {
  const double q = __dmul_rn(a, y);
  return __fma_rn(__fma_rn(-q, b, a), y, q);
}

// RN(a / b) for the time span b = BinnedTime.maxOffset(period) (86400000, 604800, 2678400 or 527050: the
// only z bounds XZ3SFC is built with, XZ3SFC.scala:27-36) and a = z - 0 in [0, b]: RN(1/b) b = 1 + d with
// |d| <= 0.42 * 2^-53 for all four, so div_span applies; a positive a below 2^-900 (where a y could lose
// bits to underflow) takes the IEEE divide.  Checked against a / b on 1.67e9 values per the four spans
// (tools/div_check.c).
__device__ __forceinline__ double div_time(double a, double b, double y) {
  if (a > 0.0 && a < 0x1p-900) return __ddiv_rn(a, b);
  return div_span(a, b, y);
}

// the level count: l1 >= g -> g, else l1 + 1 when the envelope fits the next level's 2x2 cells
// (XZ2SFC.scala:62-75), as selects.  l1 = Int.MaxValue (a zero-size envelope) is clamped before the
// power of two is formed; that branch's fits value is never used.
__device__ __forceinline__ int xz_length(int32_t l1, int g, int fits_all) {
  return l1 >= g ? g : (fits_all ? l1 + 1 : l1);
}

// XZ2SFC.index (z3/curve/XZ2SFC.scala:54-77) with normalize (:318-350), sequenceCode (:264-286).
// Branch-free in the common path: the status is a select, the out-of-range and NaN cases are clamped
// (fmin / fmax drop NaN) and computed like any other envelope, and the key is zeroed at the end.
template <bool LENIENT>
__device__ __forceinline__ uint8_t xz2_one(int g, double xmin, double ymin, double xmax, double ymax, int64_t& out) {
  const bool ordered = xmin <= xmax && ymin <= ymax;
  const bool inside = xmin >= -180.0 && xmax <= 180.0 && ymin >= -90.0 && ymax <= 90.0;
  const uint8_t st = !ordered ? (uint8_t)ST_UNORDERED : ((LENIENT || inside) ? (uint8_t)ST_OK : (uint8_t)ST_OUT_OF_BOUNDS);
  xmin = fmin(fmax(xmin, -180.0), 180.0); ymin = fmin(fmax(ymin, -90.0), 90.0);
  xmax = fmin(fmax(xmax, -180.0), 180.0); ymax = fmin(fmax(ymax, -90.0), 90.0);
  const double RX = 1.0 / 360.0, RY = 1.0 / 180.0;   // RN(1 / b), folded at compile time
  const double nxmin = div_span(__dsub_rn(xmin, -180.0), 360.0, RX);
  const double nymin = div_span(__dsub_rn(ymin, -90.0), 180.0, RY);
  const double nxmax = div_span(__dsub_rn(xmax, -180.0), 360.0, RX);
  const double nymax = div_span(__dsub_rn(ymax, -90.0), 180.0, RY);
  const double maxdim = jmax(__dsub_rn(nxmax, nxmin), __dsub_rn(nymax, nymin));
  const int32_t l1 = xz_l1(maxdim);
  const int32_t lc = l1 < g ? l1 : g;
  const double w2 = ldexp(1.0, -(lc + 1)), inv = ldexp(1.0, lc + 1);   // math.pow(0.5, l1 + 1), exact
  const int length = xz_length(l1, g, (int)xz_fits(nxmin, nxmax, w2, inv) & (int)xz_fits(nymin, nymax, w2, inv));
  const uint32_t ix = xz_cell(nxmin, length), iy = xz_cell(nymin, length);
  const uint64_t il = z2_split(ix) | (z2_split(iy) << 1);
  const uint64_t num = (il << (2 * (g - length + 1))) - (uint64_t)(__popc(ix) + 2 * __popc(iy));
  out = (st == ST_OK && length != 0) ? (int64_t)length + (int64_t)(num / 3u) : 0;
  return st;
}

// XZ3SFC.index (z3/curve/XZ3SFC.scala:53-76) with normalize (:338-380), sequenceCode (:275-304).  zhi is
// BinnedTime.maxOffset(period) (every caller), so z divides as div_time.
template <bool LENIENT>
__device__ __forceinline__ uint8_t xz3_one(int g, double zhi, double xmin, double ymin, double zmin, double xmax,
                                           double ymax, double zmax, int64_t& out) {
  const bool ordered = xmin <= xmax && ymin <= ymax && zmin <= zmax;
  const bool inside = xmin >= -180.0 && xmax <= 180.0 && ymin >= -90.0 && ymax <= 90.0 && zmin >= 0.0 && zmax <= zhi;
  const uint8_t st = !ordered ? (uint8_t)ST_UNORDERED : ((LENIENT || inside) ? (uint8_t)ST_OK : (uint8_t)ST_OUT_OF_BOUNDS);
  xmin = fmin(fmax(xmin, -180.0), 180.0); ymin = fmin(fmax(ymin, -90.0), 90.0); zmin = fmin(fmax(zmin, 0.0), zhi);
  xmax = fmin(fmax(xmax, -180.0), 180.0); ymax = fmin(fmax(ymax, -90.0), 90.0); zmax = fmin(fmax(zmax, 0.0), zhi);
  const double RX = 1.0 / 360.0, RY = 1.0 / 180.0;
  const double zsize = __dsub_rn(zhi, 0.0);
  const double nxmin = div_span(__dsub_rn(xmin, -180.0), 360.0, RX);
  const double nymin = div_span(__dsub_rn(ymin, -90.0), 180.0, RY);
  const double RZ = __ddiv_rn(1.0, zsize);   // uniform: hoisted out of the caller's loop
  const double nzmin = div_time(__dsub_rn(zmin, 0.0), zsize, RZ);
  const double nxmax = div_span(__dsub_rn(xmax, -180.0), 360.0, RX);
  const double nymax = div_span(__dsub_rn(ymax, -90.0), 180.0, RY);
  const double nzmax = div_time(__dsub_rn(zmax, 0.0), zsize, RZ);
  const double maxdim = jmax(jmax(__dsub_rn(nxmax, nxmin), __dsub_rn(nymax, nymin)), __dsub_rn(nzmax, nzmin));
  const int32_t l1 = xz_l1(maxdim);
  const int32_t lc = l1 < g ? l1 : g;
  const double w2 = ldexp(1.0, -(lc + 1)), inv = ldexp(1.0, lc + 1);
  const int length = xz_length(l1, g, (int)xz_fits(nxmin, nxmax, w2, inv) & (int)xz_fits(nymin, nymax, w2, inv) &
                                          (int)xz_fits(nzmin, nzmax, w2, inv));
  const uint32_t ix = xz_cell(nxmin, length), iy = xz_cell(nymin, length), iz = xz_cell(nzmin, length);
  const uint64_t il = z3_split(ix) | (z3_split(iy) << 1) | (z3_split(iz) << 2);
  const uint64_t num = (il << (3 * (g - length + 1))) - (uint64_t)(__popc(ix) + 2 * __popc(iy) + 4 * __popc(iz));
  out = (st == ST_OK && length != 0) ? (int64_t)length + (int64_t)(num / 7u) : 0;
  return st;
}

// ------------------------------------------------------------------ host-side dimension setup
inline bool valid_period(int p) { return p >= DAY && p <= YEAR; }

inline NDim lon_dim(int p) { return make_ndim(-180.0, 180.0, p); }
inline NDim lat_dim(int p) { return make_ndim(-90.0, 90.0, p); }
inline NDim time_dim(int period, int p) { return make_ndim(0.0, (double)max_offset(period), p); }

}  // namespace gm
