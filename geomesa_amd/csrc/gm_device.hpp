// gm_device.hpp -- device-side building blocks of the GeoMesa hot path for gfx950 (CDNA4).
//
// Everything here is __device__ code that restates the reference Scala arithmetic bit-exactly:
//   * JVM double->int/long conversions saturate (JLS 5.1.3) -- plain C++ casts are UB out of range;
//   * no multiply-add contraction (the JVM never fuses): every TU is built with -ffp-contract=off and
//     the pragma below;
//   * arithmetic (>>) vs logical (>>>) shifts follow the Scala source line by line.
// Reference paths are abbreviated  z3/ = geomesa-z3/src/main/scala/org/locationtech/geomesa/
//                                  idx/ = geomesa-index-api/src/main/scala/org/locationtech/geomesa/index/
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gm {

// clang ext-vector types: one dwordx4 per lane; usable with the nontemporal builtins
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef long long lv2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------- status codes (per element)
enum : uint8_t { ST_OK = 0, ST_OUT_OF_BOUNDS = 1, ST_BAD_TIME = 2, ST_UNORDERED = 3, ST_NULL_GEOM = 4 };
enum : int { DAY = 0, WEEK = 1, MONTH = 2, YEAR = 3 };

// ---------------------------------------------------------------- JVM conversions
// JVM d2i: NaN -> 0, saturating.  Branch-free (clamp, convert, select): the three early returns compiled
// to nested exec-mask branches, ~12 scalar instructions per conversion around ~4 vector ones, which the
// VALU-heavy kernels (Z3Histogram: three normalizations per point) paid on every point.
__device__ __forceinline__ int32_t jvm_d2i(double d) {
  const double c = __builtin_fmin(__builtin_fmax(d, -2147483648.0), 2147483647.0);   // NaN -> -2^31 here ...
  const int32_t r = (int32_t)c;                                                      // (in range: defined)
  return d == d ? r : 0;                                                             // ... and 0 here
}
__device__ __forceinline__ int64_t jvm_d2l(double d) {
  if (!(d == d)) return 0;
  if (d >= 9223372036854775808.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}

// ---------------------------------------------------------------- Z3 interleave
// Z3.split (z3/zorder/sfcurve/Z3.scala:73-80): 21 bits -> every third bit of 63.
// Done in two 32-bit halves: bits 0..10 of the input land in the low word (bits 0..30), bits 11..20
// in the high word (bits 33..60). Each half is a classic 32-bit magic-number spread, which costs
// VALU half of the 64-bit form on CDNA (64-bit logic ops issue as two 32-bit ops).
__device__ __forceinline__ uint32_t spread3_11(uint32_t x) {  // x < 2^11 -> bits at 3k
  x &= 0x7ffu;
  x = (x | (x << 16)) & 0x070000ffu;
  x = (x | (x << 8)) & 0x0700f00fu;
  x = (x | (x << 4)) & 0x430c30c3u;
  x = (x | (x << 2)) & 0x49249249u;
  return x;
}
__device__ __forceinline__ uint64_t z3_split(int64_t value) {
  uint32_t v = (uint32_t)((uint64_t)value & 0x1fffffull);
  uint32_t lo = spread3_11(v & 0x7ffu);          // input bits 0..10 -> z bits 0..30
  uint32_t hi = spread3_11(v >> 11);             // input bits 11..20 -> z bits 33..60 (= 33 + 3k)
  return ((uint64_t)hi << 33) | (uint64_t)lo;
}
// Z3.combine (Z3.scala:83-91): inverse, 21-bit result
__device__ __forceinline__ uint32_t compact3_11(uint32_t x) {
  x &= 0x49249249u;
  x = (x ^ (x >> 2)) & 0x430c30c3u;
  x = (x ^ (x >> 4)) & 0x0700f00fu;
  x = (x ^ (x >> 8)) & 0x070000ffu;
  x = (x ^ (x >> 16)) & 0x7ffu;
  return x;
}
__device__ __forceinline__ int32_t z3_combine(int64_t z) {
  uint64_t u = (uint64_t)z;
  uint32_t lo = compact3_11((uint32_t)u & 0x49249249u);            // z bits 0..30 step 3
  uint32_t hi = compact3_11((uint32_t)(u >> 33) & 0x09249249u);    // z bits 33..60 step 3 (10 bits)
  return (int32_t)(lo | (hi << 11));
}
// Z3.apply (Z3.scala:66-68) -- Int arguments widen to Long, split masks to 21 bits
__device__ __forceinline__ int64_t z3_apply(int32_t x, int32_t y, int32_t t) {
  return (int64_t)(z3_split(x) | (z3_split(y) << 1) | (z3_split(t) << 2));
}

// ---------------------------------------------------------------- Z2 interleave
// Z2.split (z3/zorder/sfcurve/Z2.scala:58-67): 31 bits -> even bits of 62. Two 16-bit halves.
__device__ __forceinline__ uint32_t spread2_16(uint32_t x) {
  x &= 0xffffu;
  x = (x | (x << 8)) & 0x00ff00ffu;
  x = (x | (x << 4)) & 0x0f0f0f0fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}
__device__ __forceinline__ uint64_t z2_split(int64_t value) {
  uint32_t v = (uint32_t)((uint64_t)value & 0x7fffffffull);
  return ((uint64_t)spread2_16(v >> 16) << 32) | (uint64_t)spread2_16(v & 0xffffu);
}
__device__ __forceinline__ uint32_t compact2_16(uint32_t x) {
  x &= 0x55555555u;
  x = (x ^ (x >> 1)) & 0x33333333u;
  x = (x ^ (x >> 2)) & 0x0f0f0f0fu;
  x = (x ^ (x >> 4)) & 0x00ff00ffu;
  x = (x ^ (x >> 8)) & 0x0000ffffu;
  return x;
}
// Z2.combine (Z2.scala:70-78): 32 result bits (bit 62 of z lands in bit 31), then .toInt
__device__ __forceinline__ int32_t z2_combine(int64_t z) {
  uint64_t u = (uint64_t)z;
  return (int32_t)(compact2_16((uint32_t)u) | (compact2_16((uint32_t)(u >> 32)) << 16));
}
__device__ __forceinline__ int64_t z2_apply(int32_t x, int32_t y) {
  return (int64_t)(z2_split(x) | (z2_split(y) << 1));
}

// ---------------------------------------------------------------- BitNormalizedDimension
// z3/curve/NormalizedDimension.scala:56-72. normalizer/denormalizer are folded at compile time in
// IEEE binary64, exactly the values the JVM computes in the constructor.
struct NDim {
  double min, max, normalizer, denormalizer;
  int32_t max_index;
};
__host__ __device__ constexpr NDim make_ndim(double mn, double mx, int precision) {
  return NDim{mn, mx, (double)(1LL << precision) / (mx - mn), (mx - mn) / (double)(1LL << precision),
              (int32_t)((1LL << precision) - 1)};
}
__device__ __forceinline__ int32_t normalize(const NDim& d, double x) {
  // a select, not a branch (see jvm_d2i)
  const int32_t r = jvm_d2i(floor(__dmul_rn(__dsub_rn(x, d.min), d.normalizer)));
  return x >= d.max ? d.max_index : r;
}
__device__ __forceinline__ double denormalize(const NDim& d, int32_t i) {
  double a = (i >= d.max_index) ? (double)d.max_index : (double)i;
  return __dadd_rn(d.min, __dmul_rn(__dadd_rn(a, 0.5), d.denormalizer));
}

// BinnedTime.maxOffset (z3/curve/BinnedTime.scala:148-156)
__host__ __device__ constexpr int64_t max_offset(int period) {
  return period == DAY ? 86400000LL : period == WEEK ? 604800LL : period == MONTH ? 86400LL * 31LL
                                                                                    : 1440LL * 366LL + 10LL;
}

// ---------------------------------------------------------------- civil calendar (java.time UTC)
__device__ __forceinline__ int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
// valid only for z >= 0 (times are rejected before the epoch)
__device__ __forceinline__ void civil_from_days(int64_t z, int64_t& y, int64_t& m) {
  z += 719468;
  int64_t era = z / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  m = mp < 10 ? mp + 3 : mp - 9;
  y = yoe + era * 400 + (m <= 2);
}

// BinnedTime.timeToBinnedTime (BinnedTime.scala:73-86, 198-277): epoch-ms -> (bin, offset).
// require(!date.isBefore(epoch)) and require(maxDate.isAfter(date)) become ST_BAD_TIME.
// Division by constants is strength-reduced by the compiler (no 64-bit divide loop).
template <int PERIOD>
__device__ __forceinline__ uint8_t binned_time(int64_t ms, int16_t& bin, int64_t& off) {
  if (ms < 0) { bin = 0; off = 0; return ST_BAD_TIME; }
  const uint64_t u = (uint64_t)ms;
  if (PERIOD == WEEK) {
    uint64_t w = u / 604800000ull;
    if (w >= 32768) { bin = 0; off = 0; return ST_BAD_TIME; }
    uint32_t r = (uint32_t)(u - w * 604800000ull);       // < 604800000 < 2^30
    bin = (int16_t)w; off = (int64_t)(r / 1000u);         // floorDiv(ms,1000) - w*604800
    return ST_OK;
  } else if (PERIOD == DAY) {
    uint64_t dd = u / 86400000ull;
    if (dd >= 32768) { bin = 0; off = 0; return ST_BAD_TIME; }
    bin = (int16_t)dd; off = (int64_t)(u - dd * 86400000ull);
    return ST_OK;
  } else {
    int64_t y, m;
    civil_from_days((int64_t)(u / 86400000ull), y, m);
    int64_t esec = (int64_t)(u / 1000ull);
    if (PERIOD == MONTH) {
      int64_t months = (y - 1970) * 12 + (m - 1);
      if (months >= 32768) { bin = 0; off = 0; return ST_BAD_TIME; }
      bin = (int16_t)months; off = esec - days_from_civil(y, m, 1) * 86400;
    } else {
      int64_t years = y - 1970;
      if (years >= 32768) { bin = 0; off = 0; return ST_BAD_TIME; }
      bin = (int16_t)years; off = (esec - days_from_civil(y, 1, 1) * 86400) / 60;
    }
    return ST_OK;
  }
}

// ---------------------------------------------------------------- double-double helpers
struct DD { double hi, lo; };
__device__ __forceinline__ DD two_sum(double a, double b) {
  double s = __dadd_rn(a, b);
  double bb = __dsub_rn(s, a);
  double e = __dadd_rn(__dsub_rn(a, __dsub_rn(s, bb)), __dsub_rn(b, bb));
  return DD{s, e};
}
__device__ __forceinline__ DD quick_two_sum(double a, double b) {
  double s = __dadd_rn(a, b);
  return DD{s, __dsub_rn(b, __dsub_rn(s, a))};
}
__device__ __forceinline__ DD two_prod(double a, double b) {
  double p = __dmul_rn(a, b);
  return DD{p, fma(a, b, -p)};  // exact product error (not a parity-path contraction)
}
__device__ __forceinline__ DD dd_add(DD a, DD b) {
  DD s = two_sum(a.hi, b.hi);
  DD t = two_sum(a.lo, b.lo);
  s.lo = __dadd_rn(s.lo, t.hi);
  s = quick_two_sum(s.hi, s.lo);
  s.lo = __dadd_rn(s.lo, t.lo);
  return quick_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ DD dd_mul(DD a, DD b) {
  DD p = two_prod(a.hi, b.hi);
  p.lo = __dadd_rn(p.lo, __dadd_rn(__dmul_rn(a.hi, b.lo), __dmul_rn(a.lo, b.hi)));
  return quick_two_sum(p.hi, p.lo);
}

// log(m) rounded once from a ~2^-100-accurate double-double, for m = 2^k (1 + x) with |x| < 2^-19.
// Used only near powers of two, where a 1-ulp error of the device log could move
// floor(log(m)/log(0.5)) across an integer.
__device__ __forceinline__ double log_near_pow2(int k, double x) {
  const DD LN2 = {0.6931471805599453094, 2.3190468138462996e-17};
  const DD THIRD = {0.33333333333333331483, 1.8503717077085942e-17};
  DD kl = dd_mul(DD{(double)k, 0.0}, LN2);
  // log1p(x) = x - x^2/2 + x^3/3 - x^4/4 + x^5/5 - x^6/6 + x^7/7
  DD X = DD{x, 0.0};
  double tail = x * (-0.25 + x * (0.2 + x * (-1.0 / 6.0 + x * (1.0 / 7.0))));  // x^4.. terms / x^3
  DD c3 = dd_add(THIRD, DD{tail, 0.0});             // 1/3 - x/4 + ...
  DD s = dd_add(DD{-0.5, 0.0}, dd_mul(X, c3));      // -1/2 + x/3 - ...
  DD l = dd_add(DD{1.0, 0.0}, dd_mul(X, s));        // 1 - x/2 + ...
  DD lp = dd_mul(X, l);
  DD r = dd_add(kl, lp);
  return __dadd_rn(r.hi, r.lo);
}

// XZ length l1 = floor(log(maxDim) / log(0.5)).toInt (z3/curve/XZ2SFC.scala:63, XZ3SFC.scala:62)
__device__ __forceinline__ int32_t xz_l1(double maxdim) {
  const double LOG_HALF = -0.6931471805599453094;  // math.log(0.5), correctly rounded
  const double NEAR = 1.9073486328125e-06;         // 2^-19
  int e;
  const double f = frexp(maxdim, &e);              // maxdim = f * 2^e, f in [0.5, 1)
  // Away from powers of two (|f - 0.5|, |1 - f| >= 2^-20) the quotient log(maxdim)/log(0.5) = -e - log2(f)
  // lies in (-e, -e + 1), at least 1.4e-6 away from either integer -- far beyond the few ulps by which
  // the JVM's rounded log and division can move it -- so its floor is exactly -e.  log(0) = -inf gives
  // +inf -> Int.MaxValue.  Both are selects; only the rare near-power-of-two envelope branches.
  const bool lo = __dsub_rn(f, 0.5) < 0.5 * NEAR, hi = __dsub_rn(1.0, f) < 0.5 * NEAR;
  int32_t r = maxdim == 0.0 ? INT32_MAX : -e;
  if (((int)lo | (int)hi) & (int)(maxdim != 0.0)) {
    // m = 2^(e-1) (2f) with 2f - 1 exact, or m = 2^e f with f - 1 exact
    const double lg = log_near_pow2(lo ? e - 1 : e, lo ? __dsub_rn(__dmul_rn(2.0, f), 1.0) : __dsub_rn(f, 1.0));
    r = jvm_d2i(floor(__ddiv_rn(lg, LOG_HALF)));
  }
  return r;
}

// ---------------------------------------------------------------- JTS orientation (CGAlgorithmsDD)
// Orientation.index -> CGAlgorithmsDD.orientationIndex: fast filter (DP_SAFE_EPSILON = 1e-15), then
// the DD determinant with Dekker split (SPLIT = 2^27+1), operation for operation as JTS 1.20 DD.java.
__device__ __forceinline__ int dsign(double x) { return x > 0.0 ? 1 : (x < 0.0 ? -1 : 0); }

__device__ __noinline__ int jts_orientation_dd(double p1x, double p1y, double p2x, double p2y,
                                               double qx, double qy) {
  // DD.valueOf(a).selfAdd(b)  (DD.selfAdd(double))
  auto add_d = [](double hi, double lo, double y, double& rhi, double& rlo) {
    double S = __dadd_rn(hi, y);
    double e = __dsub_rn(S, hi);
    double s = __dsub_rn(S, e);
    s = __dadd_rn(__dsub_rn(y, e), __dsub_rn(hi, s));
    double f = __dadd_rn(s, lo);
    double H = __dadd_rn(S, f);
    double h = __dadd_rn(f, __dsub_rn(S, H));
    rhi = __dadd_rn(H, h);
    rlo = __dadd_rn(h, __dsub_rn(H, rhi));
  };
  // DD.selfMultiply(yhi, ylo)
  auto mul = [](double hi, double lo, double yhi, double ylo, double& rhi, double& rlo) {
    const double SPLIT = 134217729.0;
    double C = __dmul_rn(SPLIT, hi);
    double hx = __dsub_rn(C, hi);
    double c = __dmul_rn(SPLIT, yhi);
    hx = __dsub_rn(C, hx);
    double tx = __dsub_rn(hi, hx);
    double hy = __dsub_rn(c, yhi);
    C = __dmul_rn(hi, yhi);
    hy = __dsub_rn(c, hy);
    double ty = __dsub_rn(yhi, hy);
    c = __dadd_rn(__dadd_rn(__dadd_rn(__dadd_rn(__dsub_rn(__dmul_rn(hx, hy), C), __dmul_rn(hx, ty)),
                                      __dmul_rn(tx, hy)),
                            __dmul_rn(tx, ty)),
                  __dadd_rn(__dmul_rn(hi, ylo), __dmul_rn(lo, yhi)));
    double zhi = __dadd_rn(C, c);
    hx = __dsub_rn(C, zhi);
    rhi = zhi;
    rlo = __dadd_rn(c, hx);
  };
  double dx1h, dx1l, dy1h, dy1l, dx2h, dx2l, dy2h, dy2l;
  add_d(p2x, 0.0, -p1x, dx1h, dx1l);
  add_d(p2y, 0.0, -p1y, dy1h, dy1l);
  add_d(qx, 0.0, -p2x, dx2h, dx2l);
  add_d(qy, 0.0, -p2y, dy2h, dy2l);
  double ah, al, bh, bl;
  mul(dx1h, dx1l, dy2h, dy2l, ah, al);
  mul(dy1h, dy1l, dx2h, dx2l, bh, bl);
  // DD.selfSubtract(b) = selfAdd(-b.hi, -b.lo)  (DD.selfAdd(double, double))
  double yhi = -bh, ylo = -bl;
  double S = __dadd_rn(ah, yhi);
  double T = __dadd_rn(al, ylo);
  double e = __dsub_rn(S, ah);
  double f = __dsub_rn(T, al);
  double s = __dsub_rn(S, e);
  double t = __dsub_rn(T, f);
  s = __dadd_rn(__dsub_rn(yhi, e), __dsub_rn(ah, s));
  t = __dadd_rn(__dsub_rn(ylo, f), __dsub_rn(al, t));
  e = __dadd_rn(s, T);
  double H = __dadd_rn(S, e);
  double h = __dadd_rn(e, __dsub_rn(S, H));
  e = __dadd_rn(t, h);
  double zhi = __dadd_rn(H, e);
  double zlo = __dadd_rn(e, __dsub_rn(H, zhi));
  if (zhi > 0.0) return 1;
  if (zhi < 0.0) return -1;
  if (zlo > 0.0) return 1;
  if (zlo < 0.0) return -1;
  return 0;
}

__device__ __forceinline__ int jts_orientation(double p1x, double p1y, double p2x, double p2y, double qx,
                                               double qy) {
  double detleft = __dmul_rn(__dsub_rn(p1x, qx), __dsub_rn(p2y, qy));
  double detright = __dmul_rn(__dsub_rn(p1y, qy), __dsub_rn(p2x, qx));
  double det = __dsub_rn(detleft, detright);
  double detsum;
  if (detleft > 0.0) {
    if (detright <= 0.0) return dsign(det);
    detsum = __dadd_rn(detleft, detright);
  } else if (detleft < 0.0) {
    if (detright >= 0.0) return dsign(det);
    detsum = __dsub_rn(-detleft, detright);
  } else {
    return dsign(det);
  }
  double errbound = __dmul_rn(1e-15, detsum);
  if ((det >= errbound) || (-det >= errbound)) return dsign(det);
  return jts_orientation_dd(p1x, p1y, p2x, p2y, qx, qy);
}

// wave compaction helpers: the number of set bits of a ballot below this lane, and a wave-scope
// ordering point for LDS written by other lanes of the same wave
__device__ __forceinline__ int lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

}  // namespace gm
