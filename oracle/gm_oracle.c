/*
 * gm_oracle.c -- TEST INFRASTRUCTURE ONLY (see gm_oracle.h).
 *
 * Scalar, bit-exact CPU restatement of the reference Scala hot path.  Compile with
 * -ffp-contract=off and without -ffast-math: the JVM never fuses multiply-add and
 * uses IEEE-754 binary64 throughout.
 */
#include "gm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

/* ------------------------------------------------------------------ */
/* JVM numeric semantics                                              */
/* ------------------------------------------------------------------ */

/* Double.toInt: NaN -> 0, saturating (JLS 5.1.3) */
int32_t gmo_d2i(double d) {
  if (d != d) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}

/* Double.toLong: NaN -> 0, saturating (JLS 5.1.3) */
int64_t gmo_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775808.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}

/* Java shift semantics: the distance is masked to 6 bits for longs */
static inline int64_t jshl(int64_t v, int s) { return (int64_t)((uint64_t)v << (s & 63)); }
static inline int64_t jshr(int64_t v, int s) { return v >> (s & 63); }             /* >>  */
static inline int64_t jushr(int64_t v, int s) { return (int64_t)((uint64_t)v >> (s & 63)); } /* >>> */

/* ------------------------------------------------------------------ */
/* Z3 / Z2 bit interleave  (z3/../zorder/sfcurve/Z3.scala:52-91, Z2.scala:43-78) */
/* ------------------------------------------------------------------ */

#define Z3_MAXMASK 0x1fffffLL
#define Z2_MAXMASK 0x7fffffffLL

/* Z3.split (Z3.scala:73-80) */
int64_t gmo_z3_split(int64_t value) {
  uint64_t x = (uint64_t)(value & Z3_MAXMASK);
  x = (x | x << 32) & 0x1f00000000ffffULL;
  x = (x | x << 16) & 0x1f0000ff0000ffULL;
  x = (x | x << 8) & 0x100f00f00f00f00fULL;
  x = (x | x << 4) & 0x10c30c30c30c30c3ULL;
  return (int64_t)((x | x << 2) & 0x1249249249249249ULL);
}

/* Z3.combine (Z3.scala:83-91) */
int32_t gmo_z3_combine(int64_t z) {
  int64_t x = z & 0x1249249249249249LL;
  x = (x ^ (x >> 2)) & 0x10c30c30c30c30c3LL;
  x = (x ^ (x >> 4)) & 0x100f00f00f00f00fLL;
  x = (x ^ (x >> 8)) & 0x1f0000ff0000ffLL;
  x = (x ^ (x >> 16)) & 0x1f00000000ffffLL;
  x = (x ^ (x >> 32)) & Z3_MAXMASK;
  return (int32_t)(uint32_t)(uint64_t)x;
}

/* Z3.apply(x, y, z) (Z3.scala:66-68); Int arguments widen to Long (sign-extended) */
int64_t gmo_z3_apply(int32_t x, int32_t y, int32_t t) {
  return gmo_z3_split(x) | jshl(gmo_z3_split(y), 1) | jshl(gmo_z3_split(t), 2);
}

/* Z2.split (Z2.scala:58-67) */
int64_t gmo_z2_split(int64_t value) {
  uint64_t x = (uint64_t)(value & Z2_MAXMASK);
  x = (x ^ (x << 32)) & 0x00000000ffffffffULL;
  x = (x ^ (x << 16)) & 0x0000ffff0000ffffULL;
  x = (x ^ (x << 8)) & 0x00ff00ff00ff00ffULL;
  x = (x ^ (x << 4)) & 0x0f0f0f0f0f0f0f0fULL;
  x = (x ^ (x << 2)) & 0x3333333333333333ULL;
  x = (x ^ (x << 1)) & 0x5555555555555555ULL;
  return (int64_t)x;
}

/* Z2.combine (Z2.scala:70-78); final .toInt keeps the low 32 bits */
int32_t gmo_z2_combine(int64_t z) {
  int64_t x = z & 0x5555555555555555LL;
  x = (x ^ (x >> 1)) & 0x3333333333333333LL;
  x = (x ^ (x >> 2)) & 0x0f0f0f0f0f0f0f0fLL;
  x = (x ^ (x >> 4)) & 0x00ff00ff00ff00ffLL;
  x = (x ^ (x >> 8)) & 0x0000ffff0000ffffLL;
  x = (x ^ (x >> 16)) & 0x00000000ffffffffLL;
  return (int32_t)(uint32_t)(uint64_t)x;
}

/* Z2.apply (Z2.scala:53) */
int64_t gmo_z2_apply(int32_t x, int32_t y) { return gmo_z2_split(x) | jshl(gmo_z2_split(y), 1); }

/* per-dimension decode, d0/d1/d2 (Z3.scala:22-24, Z2.scala:26-31) */
static inline int32_t zdim(int dims, int64_t z, int d) {
  return dims == 3 ? gmo_z3_combine(jshr(z, d)) : gmo_z2_combine(jshr(z, d));
}
static inline int64_t zsplit(int dims, int64_t v) { return dims == 3 ? gmo_z3_split(v) : gmo_z2_split(v); }

/* Z3.contains / Z2.contains (Z3.scala:93-98, Z2.scala:80-83) */
int gmo_zn_contains(int dims, int64_t rmin, int64_t rmax, int64_t value) {
  for (int d = 0; d < dims; d++) {
    int32_t v = zdim(dims, value, d);
    if (!(v >= zdim(dims, rmin, d) && v <= zdim(dims, rmax, d))) return 0;
  }
  return 1;
}

/* Z3.overlaps / Z2.overlaps (Z3.scala:100-105, Z2.scala:85-89) */
int gmo_zn_overlaps(int dims, int64_t rmin, int64_t rmax, int64_t vmin, int64_t vmax) {
  for (int d = 0; d < dims; d++) {
    int32_t a1 = zdim(dims, rmin, d), a2 = zdim(dims, rmax, d);
    int32_t b1 = zdim(dims, vmin, d), b2 = zdim(dims, vmax, d);
    int32_t lo = a1 > b1 ? a1 : b1, hi = a2 < b2 ? a2 : b2;
    if (!(lo <= hi)) return 0;
  }
  return 1;
}

/* ZN.load (ZN.scala:284-288) */
static int64_t zn_load(int dims, int64_t target, int64_t p, int bits, int dim) {
  int bpd = dims == 3 ? 21 : 31;
  int64_t maxmask = dims == 3 ? Z3_MAXMASK : Z2_MAXMASK;
  int64_t mask = ~jshl(zsplit(dims, jshr(maxmask, bpd - bits)), dim);
  int64_t wiped = target & mask;
  return wiped | jshl(zsplit(dims, p), dim);
}

/* ZN.zdiv, Tropf LITMAX/BIGMIN (ZN.scala:309-361) */
void gmo_zdivide(int dims, int64_t xd, int64_t rmin, int64_t rmax, int64_t* litmax_out, int64_t* bigmin_out) {
  int64_t zmin = rmin, zmax = rmax, bigmin = 0, litmax = 0;
  for (int i = 63; i >= 0; i--) {
    int bits = i / dims + 1, dim = i % dims;
    int bx = (int)jshr(xd & jshl(1, i), i), bmn = (int)jshr(zmin & jshl(1, i), i), bmx = (int)jshr(zmax & jshl(1, i), i);
    int64_t over = jshl(1, bits - 1), under = jshl(1, bits - 1) - 1;
    int key = (bx & 1) << 2 | (bmn & 1) << 1 | (bmx & 1);
    switch (key) {
      case 1: /* (0,0,1) */
        zmax = zn_load(dims, zmax, under, bits, dim);
        bigmin = zn_load(dims, zmin, over, bits, dim);
        break;
      case 3: /* (0,1,1) */
        *litmax_out = litmax; *bigmin_out = zmin; return;
      case 4: /* (1,0,0) */
        *litmax_out = zmax; *bigmin_out = bigmin; return;
      case 5: /* (1,0,1) */
        litmax = zn_load(dims, zmax, under, bits, dim);
        zmin = zn_load(dims, zmin, over, bits, dim);
        break;
      default: break; /* (0,0,0), (1,1,1) continue; (0,1,0), (1,1,0) impossible */
    }
  }
  *litmax_out = litmax; *bigmin_out = bigmin;
}

/* ZN.longestCommonPrefix (ZN.scala:272-281) */
void gmo_longest_common_prefix(int dims, const int64_t* values, int n, int64_t* prefix, int* bits) {
  int total = dims == 3 ? 63 : 62;
  int shift = total - dims;
  int64_t head = jushr(values[0], shift);
  for (;;) {
    int all = 1;
    for (int i = 1; i < n; i++) if (jushr(values[i], shift) != head) { all = 0; break; }
    if (!(all && shift > -1)) break;
    shift -= dims;
    head = jushr(values[0], shift);
  }
  shift += dims;
  *prefix = values[0] & jshl(INT64_MAX, shift);
  *bits = 64 - shift;
}

/* ---------------- growable containers ---------------- */
typedef struct { gmo_range* v; int64_t n, cap; } rvec;
static void rvec_push(rvec* r, int64_t lo, int64_t hi, int contained) {
  if (r->n == r->cap) { r->cap = r->cap ? r->cap * 2 : 128; r->v = (gmo_range*)realloc(r->v, (size_t)r->cap * sizeof(gmo_range)); }
  r->v[r->n].lower = lo; r->v[r->n].upper = hi; r->v[r->n].contained = contained; r->v[r->n].pad = 0; r->n++;
}

typedef struct { int64_t a, b; int term; } zq_item;
typedef struct { zq_item* v; int64_t head, tail, cap; } zqueue;
static void zq_push(zqueue* q, int64_t a, int64_t b, int term) {
  if (q->tail == q->cap) {
    if (q->head > 0 && q->head >= q->cap / 2) {
      memmove(q->v, q->v + q->head, (size_t)(q->tail - q->head) * sizeof(zq_item));
      q->tail -= q->head; q->head = 0;
    } else {
      q->cap = q->cap ? q->cap * 2 : 256; q->v = (zq_item*)realloc(q->v, (size_t)q->cap * sizeof(zq_item));
    }
  }
  q->v[q->tail].a = a; q->v[q->tail].b = b; q->v[q->tail].term = term; q->tail++;
}
static inline int64_t zq_size(const zqueue* q) { return q->tail - q->head; }

/* IndexRange ordering (z3/../zorder/sfcurve/package.scala:60-69) */
static int range_cmp(const void* pa, const void* pb) {
  const gmo_range* a = (const gmo_range*)pa; const gmo_range* b = (const gmo_range*)pb;
  if (a->lower != b->lower) return a->lower < b->lower ? -1 : 1;
  if (a->upper != b->upper) return a->upper < b->upper ? -1 : 1;
  return 0;
}

/* sort + merge (ZN.scala:221-241, XZ2SFC.scala:231-249). java.util.List.sort is a stable merge
   sort; equal (lower, upper) keys only differ in `contained`, and merging AND-combines them in
   order, so stability is irrelevant to the merged output except for exact duplicates, which AND
   commutatively. */
static int64_t sort_merge(rvec* r, gmo_range* out, int64_t cap) {
  if (r->n == 0) return 0;
  qsort(r->v, (size_t)r->n, sizeof(gmo_range), range_cmp);
  int64_t m = 0;
  gmo_range cur = r->v[0];
  for (int64_t i = 1; i < r->n; i++) {
    gmo_range x = r->v[i];
    int64_t up1 = (int64_t)((uint64_t)cur.upper + 1u); /* Java long wraps */
    if (x.lower <= up1) {
      cur.upper = cur.upper > x.upper ? cur.upper : x.upper;
      cur.contained = cur.contained && x.contained;
    } else {
      if (m < cap) out[m] = cur;
      m++;
      cur = x;
    }
  }
  if (m < cap) out[m] = cur;
  m++;
  return m <= cap ? m : -m;
}

/* tree nodes checked by the range decompositions on this thread (ZN.checkValue calls, XZ elements
   tested for containment / overlap): the work measure of SURVEY 8(d)'s ranges() row */
static __thread int64_t g_nodes_checked;

int64_t gmo_nodes_checked(void) {
  const int64_t v = g_nodes_checked;
  g_nodes_checked = 0;
  return v;
}

/* ZN.zranges (ZN.scala:110-242) */
int64_t gmo_zranges(int dims, const int64_t* bounds, int nb, int precision, int max_ranges,
                    int max_recurse, gmo_range* out, int64_t cap) {
  if (nb <= 0) return 0;
  rvec ranges = {0};
  zqueue q = {0};
  int64_t* vals = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)nb);
  for (int i = 0; i < nb; i++) { vals[2 * i] = bounds[2 * i]; vals[2 * i + 1] = bounds[2 * i + 1]; }
  int64_t prefix; int common;
  gmo_longest_common_prefix(dims, vals, 2 * nb, &prefix, &common);
  free(vals);
  int offset = 64 - common;
  const int quadrants = 1 << dims;

#define IS_CONTAINED(mn, mx, res) do { res = 0; for (int _i = 0; _i < nb; _i++) \
    if (gmo_zn_contains(dims, bounds[2*_i], bounds[2*_i+1], mn) && gmo_zn_contains(dims, bounds[2*_i], bounds[2*_i+1], mx)) { res = 1; break; } } while (0)
#define IS_OVERLAPPED(mn, mx, res) do { res = 0; for (int _i = 0; _i < nb; _i++) \
    if (gmo_zn_overlaps(dims, bounds[2*_i], bounds[2*_i+1], mn, mx)) { res = 1; break; } } while (0)
#define CHECK_VALUE(pfx, quad) do { \
    g_nodes_checked++; \
    int64_t _mn = (pfx) | jshl((quad), offset); \
    int64_t _mx = _mn | (jshl(1, offset) - 1); \
    int _c; IS_CONTAINED(_mn, _mx, _c); \
    if (_c || offset < 64 - precision) rvec_push(&ranges, _mn, _mx, 1); \
    else { int _o; IS_OVERLAPPED(_mn, _mx, _o); if (_o) zq_push(&q, _mn, _mx, 0); } } while (0)
#define BOTTOM_OUT() do { do { zq_item _it = q.v[q.head++]; \
    if (!_it.term) rvec_push(&ranges, _it.a, _it.b, 0); } while (zq_size(&q) > 0); } while (0)

  CHECK_VALUE(prefix, (int64_t)0);
  zq_push(&q, -1, -1, 1);
  offset -= dims;
  int level = 0;
  const int64_t range_stop = max_ranges;
  const int recurse_stop = max_recurse;
  do {
    zq_item next = q.v[q.head++];
    if (next.term) {
      if (zq_size(&q) > 0) {
        level += 1;
        offset -= dims;
        if (level >= recurse_stop || offset < 0) BOTTOM_OUT();
        else zq_push(&q, -1, -1, 1);
      }
    } else {
      int64_t pfx = next.a;
      for (int64_t quad = 0; quad < quadrants; quad++) CHECK_VALUE(pfx, quad);
      if (ranges.n + zq_size(&q) - 1 >= range_stop) BOTTOM_OUT();
    }
  } while (zq_size(&q) > 0);
#undef IS_CONTAINED
#undef IS_OVERLAPPED
#undef CHECK_VALUE
#undef BOTTOM_OUT
  free(q.v);
  int64_t m = sort_merge(&ranges, out, cap);
  free(ranges.v);
  return m;
}

/* ------------------------------------------------------------------ */
/* NormalizedDimension (z3/curve/NormalizedDimension.scala:56-78)      */
/* ------------------------------------------------------------------ */

int32_t gmo_normalize(double min, double max, int precision, double x) {
  int64_t bins = (int64_t)1 << precision;
  double normalizer = (double)bins / (max - min);
  int32_t max_index = (int32_t)(bins - 1);
  if (x >= max) return max_index;
  double v = (x - min) * normalizer;
  return gmo_d2i(floor(v));
}

double gmo_denormalize(double min, double max, int precision, int32_t i) {
  int64_t bins = (int64_t)1 << precision;
  double denormalizer = (max - min) / (double)bins;
  int32_t max_index = (int32_t)(bins - 1);
  if (i >= max_index) { double a = (double)max_index + 0.5; double b = a * denormalizer; return min + b; }
  double a = (double)i + 0.5; double b = a * denormalizer; return min + b;
}

/* ------------------------------------------------------------------ */
/* BinnedTime (z3/curve/BinnedTime.scala)                              */
/* ------------------------------------------------------------------ */

/* BinnedTime.maxOffset (BinnedTime.scala:148-156) */
int64_t gmo_max_offset(int period) {
  switch (period) {
    case GMO_DAY: return 86400000LL;
    case GMO_WEEK: return 604800LL;
    case GMO_MONTH: return 86400LL * 31LL;
    case GMO_YEAR: return 1440LL * 366LL + 10LL;
  }
  return 0;
}

static int64_t floor_div(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) q--; return q; }

/* proleptic Gregorian civil date <-> epoch day (java.time.LocalDate semantics) */
static int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
static void civil_from_days(int64_t z, int64_t* y, int64_t* m, int64_t* d) {
  z += 719468;
  int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t yy = yoe + era * 400;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  *d = doy - (153 * mp + 2) / 5 + 1;
  *m = mp < 10 ? mp + 3 : mp - 9;
  *y = yy + (*m <= 2);
}

/* timeToBinnedTime: toDayAndMillis / toWeekAndSeconds / toMonthAndSeconds / toYearAndMinutes
   (BinnedTime.scala:198-277). require(!before epoch) and require(maxDate after date). */
int gmo_binned_time(int period, int64_t ms, int16_t* bin, int64_t* offset) {
  *bin = 0; *offset = 0;
  if (ms < 0) return GMO_BAD_TIME;
  int64_t esec = floor_div(ms, 1000);
  switch (period) {
    case GMO_DAY: {
      int64_t days = ms / 86400000LL;
      if (days >= 32768) return GMO_BAD_TIME;
      *bin = (int16_t)days; *offset = ms - days * 86400000LL; return GMO_OK;
    }
    case GMO_WEEK: {
      int64_t weeks = ms / 604800000LL;
      if (weeks >= 32768) return GMO_BAD_TIME;
      *bin = (int16_t)weeks; *offset = esec - weeks * 604800LL; return GMO_OK;
    }
    case GMO_MONTH: {
      int64_t y, m, d; civil_from_days(ms / 86400000LL, &y, &m, &d);
      int64_t months = (y - 1970) * 12 + (m - 1);
      if (months >= 32768) return GMO_BAD_TIME;
      int64_t start = days_from_civil(y, m, 1) * 86400LL;
      *bin = (int16_t)months; *offset = esec - start; return GMO_OK;
    }
    case GMO_YEAR: {
      int64_t y, m, d; civil_from_days(ms / 86400000LL, &y, &m, &d);
      int64_t years = y - 1970;
      if (years >= 32768) return GMO_BAD_TIME;
      int64_t start = days_from_civil(y, 1, 1) * 86400LL;
      *bin = (int16_t)years; *offset = (esec - start) / 60; return GMO_OK;
    }
  }
  return GMO_BAD_TIME;
}

/* binnedTimeToDate (BinnedTime.scala:216-280), as epoch millis */
int64_t gmo_binned_to_millis(int period, int16_t bin, int64_t offset) {
  switch (period) {
    case GMO_DAY: return (int64_t)bin * 86400000LL + offset;
    case GMO_WEEK: return (int64_t)bin * 604800000LL + offset * 1000LL;
    case GMO_MONTH: {
      int64_t mi = 1970 * 12 + (int64_t)bin; int64_t y = floor_div(mi, 12), m = mi - y * 12 + 1;
      return days_from_civil(y, m, 1) * 86400000LL + offset * 1000LL;
    }
    case GMO_YEAR: return days_from_civil(1970 + (int64_t)bin, 1, 1) * 86400000LL + offset * 60000LL;
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* Z3SFC / Z2SFC (z3/curve/Z3SFC.scala:37-67, Z2SFC.scala:26-52)     */
/* ------------------------------------------------------------------ */

int gmo_z3_index(int period, int precision, double x, double y, int64_t t, int lenient, int64_t* z) {
  const double tmax = (double)gmo_max_offset(period);
  double td = (double)t;
  if (!(x >= -180.0 && x <= 180.0 && y >= -90.0 && y <= 90.0 && td >= 0.0 && td <= tmax)) {
    if (!lenient) { *z = 0; return GMO_OUT_OF_BOUNDS; }
    /* lenientIndex (Z3SFC.scala:47-52): NaN passes through the clamps */
    x = x < -180.0 ? -180.0 : (x > 180.0 ? 180.0 : x);
    y = y < -90.0 ? -90.0 : (y > 90.0 ? 90.0 : y);
    t = td < 0.0 ? 0 : (td > tmax ? (int64_t)tmax : t);   /* bt: Long (time.min/max .toLong) */
    td = (double)t;
  }
  *z = gmo_z3_apply(gmo_normalize(-180.0, 180.0, precision, x), gmo_normalize(-90.0, 90.0, precision, y),
                    gmo_normalize(0.0, tmax, precision, td));
  return GMO_OK;
}

void gmo_z3_invert(int period, int precision, int64_t z, double* x, double* y, int64_t* t) {
  const double tmax = (double)gmo_max_offset(period);
  *x = gmo_denormalize(-180.0, 180.0, precision, gmo_z3_combine(z));
  *y = gmo_denormalize(-90.0, 90.0, precision, gmo_z3_combine(jshr(z, 1)));
  *t = gmo_d2l(gmo_denormalize(0.0, tmax, precision, gmo_z3_combine(jshr(z, 2))));
}

int gmo_z2_index(int precision, double x, double y, int lenient, int64_t* z) {
  if (!(x >= -180.0 && x <= 180.0 && y >= -90.0 && y <= 90.0)) {
    if (!lenient) { *z = 0; return GMO_OUT_OF_BOUNDS; }
    x = x < -180.0 ? -180.0 : (x > 180.0 ? 180.0 : x);
    y = y < -90.0 ? -90.0 : (y > 90.0 ? 90.0 : y);
  }
  *z = gmo_z2_apply(gmo_normalize(-180.0, 180.0, precision, x), gmo_normalize(-90.0, 90.0, precision, y));
  return GMO_OK;
}

void gmo_z2_invert(int precision, int64_t z, double* x, double* y) {
  *x = gmo_denormalize(-180.0, 180.0, precision, gmo_z2_combine(z));
  *y = gmo_denormalize(-90.0, 90.0, precision, gmo_z2_combine(jshr(z, 1)));
}

/* Z3IndexKeySpace.toIndexKey lines 71-76 (idx/index/z3/Z3IndexKeySpace.scala):
   BinnedTime first (throws even when lenient), then sfc.index(x, y, offset, lenient). */
void gmo_z3_index_key_batch(int period, const double* x, const double* y, const int64_t* t_ms, int64_t n,
                            int lenient, int16_t* bin, int64_t* z, uint8_t* status) {
  for (int64_t i = 0; i < n; i++) {
    int16_t b; int64_t off, zz = 0;
    int st = gmo_binned_time(period, t_ms[i], &b, &off);
    if (st == GMO_OK) st = gmo_z3_index(period, 21, x[i], y[i], off, lenient, &zz);
    if (st != GMO_OK) { b = 0; zz = 0; }
    bin[i] = b; z[i] = zz; if (status) status[i] = (uint8_t)st;
  }
}

/* ---- legacy curves: LegacyZ3SFC (curve/LegacyZ3SFC.scala:18-49), LegacyZ2SFC (LegacyZ2SFC.scala:14-26),
   LegacyYearZ3SFC (LegacyYearZ3SFC.scala:17-46); SemiNormalizedDimension (NormalizedDimension.scala:83-87) */
static int32_t semi_norm(double mn, double mx, double prec, double x) { return gmo_d2i(ceil((x - mn) / (mx - mn) * prec)); }
static int32_t semi_len(double mn, double mx, double prec, double x) {
  double c = ceil((x - mn) / (mx - mn) * prec);
  double m = (c != c) ? c : (mn >= c ? mn : c);            /* java.lang.Math.max: NaN wins */
  return gmo_d2i(m);
}
static double semi_denorm(double mn, double mx, double prec, int32_t i) {
  return i == 0 ? mn : ((double)i - 0.5) * (mx - mn) / prec + mn;
}
#define LZ_P21 2097151.0
#define LZ_P20 1048575.0
#define LZ_P31 2147483647.0

int gmo_legacy_z3_index(int period, double x, double y, int64_t t, int lenient, int64_t* z) {
  double tmax = (double)gmo_max_offset(period), td = (double)t;
  if (x >= -180.0 && x <= 180.0 && y >= -90.0 && y <= 90.0 && td >= 0.0 && td <= tmax) {
    *z = gmo_z3_apply(semi_norm(-180, 180, LZ_P21, x), semi_norm(-90, 90, LZ_P21, y), semi_norm(0, tmax, LZ_P20, td));
    return GMO_OK;
  }
  if (!lenient) { *z = 0; return GMO_OUT_OF_BOUNDS; }
  *z = gmo_z3_apply(semi_len(-180, 180, LZ_P21, x), semi_len(-90, 90, LZ_P21, y), semi_len(0, tmax, LZ_P20, td));
  return GMO_OK;
}

void gmo_legacy_z3_invert(int period, int64_t z, double* x, double* y, int64_t* t) {
  double tmax = (double)gmo_max_offset(period);
  *x = semi_denorm(-180, 180, LZ_P21, gmo_z3_combine(z));
  *y = semi_denorm(-90, 90, LZ_P21, gmo_z3_combine(jshr(z, 1)));
  *t = gmo_d2l(semi_denorm(0, tmax, LZ_P20, gmo_z3_combine(jshr(z, 2))));
}

int gmo_legacy_z2_index(double x, double y, int lenient, int64_t* z) {
  if (x >= -180.0 && x <= 180.0 && y >= -90.0 && y <= 90.0) {
    *z = gmo_z2_apply(semi_norm(-180, 180, LZ_P31, x), semi_norm(-90, 90, LZ_P31, y));
    return GMO_OK;
  }
  if (!lenient) { *z = 0; return GMO_OUT_OF_BOUNDS; }
  *z = gmo_z2_apply(semi_len(-180, 180, LZ_P31, x), semi_len(-90, 90, LZ_P31, y));
  return GMO_OK;
}

void gmo_legacy_z2_invert(int64_t z, double* x, double* y) {
  *x = semi_denorm(-180, 180, LZ_P31, gmo_z2_combine(z));
  *y = semi_denorm(-90, 90, LZ_P31, gmo_z2_combine(jshr(z, 1)));
}

/* LegacyYearZ3SFC.index: Z3SFC.index over (lon 21, lat 21, NormalizedTime(21, 52 weeks in minutes)) */
int gmo_legacy_year_z3_index(double x, double y, int64_t t, int lenient, int64_t* z) {
  const double tmax = 7.0 * 24 * 60 * 52;
  if ((double)t > tmax && t <= gmo_max_offset(3)) t = (int64_t)tmax;
  double td = (double)t;
  if (!(x >= -180.0 && x <= 180.0 && y >= -90.0 && y <= 90.0 && td >= 0.0 && td <= tmax)) {
    if (!lenient) { *z = 0; return GMO_OUT_OF_BOUNDS; }
    x = x < -180.0 ? -180.0 : (x > 180.0 ? 180.0 : x);
    y = y < -90.0 ? -90.0 : (y > 90.0 ? 90.0 : y);
    td = td < 0.0 ? 0.0 : (td > tmax ? tmax : td);
  }
  *z = gmo_z3_apply(gmo_normalize(-180.0, 180.0, 21, x), gmo_normalize(-90.0, 90.0, 21, y),
                    gmo_normalize(0.0, tmax, 21, td));
  return GMO_OK;
}

/* LongBinning.directIndex (utils/stats/BinnedArray.scala:185-201): binSize = (max - min).toDouble / length,
   i = floor((value - min) / binSize).toInt; the upper bound maps to length - 1. */
int gmo_long_binning_index(int64_t min, int64_t max, int length, int64_t v) {
  if (v < min || v > max) return -1;
  double bs = (double)(int64_t)((uint64_t)max - (uint64_t)min) / (double)length;
  double q = floor((double)(int64_t)((uint64_t)v - (uint64_t)min) / bs);
  int i = q != q ? 0 : (q >= 2147483647.0 ? 2147483647 : (q <= -2147483648.0 ? (-2147483647 - 1) : (int)q));
  if (i < 0 || i > length) return -1;
  return i == length ? length - 1 : i;
}

/* Z3Histogram.observe / unobserve (utils/stats/Z3Histogram.scala:101-128) over point features, one
   feature at a time in input order.  toKey (:80-86): BinnedTime then Z3SFC(period).index(x, y, offset,
   lenient) with lenient only for unobserve; a throwing toKey skips the feature (tally[0]).  minZ / maxZ
   (:53-54) are the z of (-180, -90, time.min) and (180, 90, time.max).  counts is binMap as a dense
   [n_bins][length] block for time bins bin_lo.., present[] its key set; other bins go to tally[1]. */
void gmo_z3_histogram(int period, const double* x, const double* y, const int64_t* t_ms, int64_t n, int length,
                      int unobserve, int bin_lo, int n_bins, uint8_t* present, int64_t* counts, int64_t* tally) {
  int64_t zmin = 0, zmax = 0;
  gmo_z3_index(period, 21, -180.0, -90.0, 0, 0, &zmin);
  gmo_z3_index(period, 21, 180.0, 90.0, gmo_max_offset(period), 0, &zmax);
  for (int64_t i = 0; i < n; i++) {
    int16_t b; int64_t off, z = 0;
    int st = gmo_binned_time(period, t_ms[i], &b, &off);
    if (st == GMO_OK) st = gmo_z3_index(period, 21, x[i], y[i], off, unobserve, &z);
    if (st != GMO_OK) { tally[0]++; continue; }
    int rb = (int)b - bin_lo;
    if (rb < 0 || rb >= n_bins) { tally[1]++; continue; }
    if (unobserve && !present[rb]) continue;
    if (!unobserve) present[rb] = 1;
    int k = gmo_long_binning_index(zmin, zmax, length, z);
    if (k >= 0) counts[(int64_t)rb * length + k] += unobserve ? -1 : 1;
  }
}

void gmo_z2_index_batch(const double* x, const double* y, int64_t n, int lenient, int64_t* z, uint8_t* status) {
  for (int64_t i = 0; i < n; i++) {
    int64_t zz; int st = gmo_z2_index(31, x[i], y[i], lenient, &zz);
    z[i] = zz; if (status) status[i] = (uint8_t)st;
  }
}

void gmo_z3_invert_batch(int period, const int64_t* z, int64_t n, double* x, double* y, int64_t* t) {
  for (int64_t i = 0; i < n; i++) gmo_z3_invert(period, 21, z[i], &x[i], &y[i], &t[i]);
}
void gmo_z2_invert_batch(const int64_t* z, int64_t n, double* x, double* y) {
  for (int64_t i = 0; i < n; i++) gmo_z2_invert(31, z[i], &x[i], &y[i]);
}

/* Z3SFC.ranges (Z3SFC.scala:59-67): index(...) is NOT lenient; Z3SFC.MaxRecursion = Int.MaxValue */
int64_t gmo_z3_ranges(int period, int precision, const double* xy, int nxy, const int64_t* t, int nt,
                      int range_precision, int max_ranges, gmo_range* out, int64_t cap) {
  int nb = nxy * nt;
  int64_t* zb = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(nb > 0 ? nb : 1));
  int k = 0;
  for (int i = 0; i < nxy; i++)
    for (int j = 0; j < nt; j++) {
      int64_t lo, hi;
      if (gmo_z3_index(period, precision, xy[4 * i], xy[4 * i + 1], t[2 * j], 0, &lo) ||
          gmo_z3_index(period, precision, xy[4 * i + 2], xy[4 * i + 3], t[2 * j + 1], 0, &hi)) {
        free(zb); return INT64_MIN + GMO_OUT_OF_BOUNDS;
      }
      if (lo > hi) { free(zb); return INT64_MIN + GMO_UNORDERED; }  /* ZRange require (package.scala:24) */
      zb[2 * k] = lo; zb[2 * k + 1] = hi; k++;
    }
  int64_t r = gmo_zranges(3, zb, nb, range_precision, max_ranges, INT32_MAX, out, cap);
  free(zb);
  return r;
}

/* Z2SFC.ranges (Z2SFC.scala:47-52): Z2.zranges with default maxRecurse = Some(7) (ZN.scala:113,293) */
int64_t gmo_z2_ranges(int precision, const double* xy, int nxy, int range_precision, int max_ranges,
                      gmo_range* out, int64_t cap) {
  int64_t* zb = (int64_t*)malloc(sizeof(int64_t) * 2 * (size_t)(nxy > 0 ? nxy : 1));
  for (int i = 0; i < nxy; i++) {
    int64_t lo, hi;
    if (gmo_z2_index(precision, xy[4 * i], xy[4 * i + 1], 0, &lo) ||
        gmo_z2_index(precision, xy[4 * i + 2], xy[4 * i + 3], 0, &hi)) { free(zb); return INT64_MIN + GMO_OUT_OF_BOUNDS; }
    if (lo > hi) { free(zb); return INT64_MIN + GMO_UNORDERED; }
    zb[2 * i] = lo; zb[2 * i + 1] = hi;
  }
  int64_t r = gmo_zranges(2, zb, nxy, range_precision, max_ranges, 7, out, cap);
  free(zb);
  return r;
}

/* ------------------------------------------------------------------ */
/* XZ2SFC / XZ3SFC (z3/curve/XZ2SFC.scala, XZ3SFC.scala)               */
/* ------------------------------------------------------------------ */

static int64_t ipow(int64_t b, int e) { int64_t r = 1; while (e-- > 0) r *= b; return r; }

/* XZSFC.LogPointFive = math.log(0.5) (XZSFC.scala:15) */
static double log_point_five(void) { return log(0.5); }

/* l1 / length computation shared by XZ2SFC.index:60-74 and XZ3SFC.index:59-73 */
static int xz_length(int g, double maxdim, const double* mins, const double* maxs, int dims) {
  int32_t l1 = gmo_d2i(floor(log(maxdim) / log_point_five()));
  if (l1 >= g) return g;
  double w2 = pow(0.5, (double)(l1 + 1));
  for (int d = 0; d < dims; d++) {
    double start = floor(mins[d] / w2) * w2;
    if (!(maxs[d] <= start + (2 * w2))) return l1;
  }
  return l1 + 1;
}

/* XZ2SFC.sequenceCode (XZ2SFC.scala:264-286) */
static int64_t xz2_seqcode(int g, double x, double y, int length) {
  double xmin = 0.0, ymin = 0.0, xmax = 1.0, ymax = 1.0;
  int64_t cs = 0;
  for (int i = 0; i < length; i++) {
    double xc = (xmin + xmax) / 2.0, yc = (ymin + ymax) / 2.0;
    int64_t step = (ipow(4, g - i) - 1) / 3;
    int q = (x < xc ? 0 : 1) + (y < yc ? 0 : 2);
    cs += 1 + (int64_t)q * step;
    if (x < xc) xmax = xc; else xmin = xc;
    if (y < yc) ymax = yc; else ymin = yc;
  }
  return cs;
}

/* XZ3SFC.sequenceCode (XZ3SFC.scala:275-304) */
static int64_t xz3_seqcode(int g, double x, double y, double z, int length) {
  double xmin = 0.0, ymin = 0.0, zmin = 0.0, xmax = 1.0, ymax = 1.0, zmax = 1.0;
  int64_t cs = 0;
  for (int i = 0; i < length; i++) {
    double xc = (xmin + xmax) / 2.0, yc = (ymin + ymax) / 2.0, zc = (zmin + zmax) / 2.0;
    int64_t step = (ipow(8, g - i) - 1) / 7;
    int q = (x < xc ? 0 : 1) + (y < yc ? 0 : 2) + (z < zc ? 0 : 4);
    cs += 1 + (int64_t)q * step;
    if (x < xc) xmax = xc; else xmin = xc;
    if (y < yc) ymax = yc; else ymin = yc;
    if (z < zc) zmax = zc; else zmin = zc;
  }
  return cs;
}

static inline double clampd(double v, double lo, double hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline double jmax(double a, double b) { /* java.lang.Math.max(double,double) */
  if (a != a) return a;
  if (a == 0.0 && b == 0.0) return signbit(a) ? b : a;
  return a >= b ? a : b;
}

/* XZ2SFC.normalize (XZ2SFC.scala:318-350) with bounds (-180,180),(-90,90) */
static int xz2_normalize(double xmin, double ymin, double xmax, double ymax, int lenient, double* n) {
  if (!(xmin <= xmax && ymin <= ymax)) return GMO_UNORDERED;
  if (!(xmin >= -180.0 && xmax <= 180.0 && ymin >= -90.0 && ymax <= 90.0)) {
    if (!lenient) return GMO_OUT_OF_BOUNDS;
    xmin = clampd(xmin, -180.0, 180.0); ymin = clampd(ymin, -90.0, 90.0);
    xmax = clampd(xmax, -180.0, 180.0); ymax = clampd(ymax, -90.0, 90.0);
  }
  n[0] = (xmin - -180.0) / 360.0; n[1] = (ymin - -90.0) / 180.0;
  n[2] = (xmax - -180.0) / 360.0; n[3] = (ymax - -90.0) / 180.0;
  return GMO_OK;
}

/* XZ2SFC.index (XZ2SFC.scala:54-77) */
int gmo_xz2_index(int g, double xmin, double ymin, double xmax, double ymax, int lenient, int64_t* out) {
  double n[4];
  int st = xz2_normalize(xmin, ymin, xmax, ymax, lenient, n);
  if (st) { *out = 0; return st; }
  double maxdim = jmax(n[2] - n[0], n[3] - n[1]);
  double mins[2] = {n[0], n[1]}, maxs[2] = {n[2], n[3]};
  int length = xz_length(g, maxdim, mins, maxs, 2);
  *out = xz2_seqcode(g, n[0], n[1], length);
  return GMO_OK;
}

/* XZ3SFC.normalize (XZ3SFC.scala:338-380), z bounds (0, maxOffset(period)) */
static int xz3_normalize(int period, double xmin, double ymin, double zmin, double xmax, double ymax, double zmax,
                         int lenient, double* n) {
  const double zhi = (double)gmo_max_offset(period);
  if (!(xmin <= xmax && ymin <= ymax && zmin <= zmax)) return GMO_UNORDERED;
  if (!(xmin >= -180.0 && xmax <= 180.0 && ymin >= -90.0 && ymax <= 90.0 && zmin >= 0.0 && zmax <= zhi)) {
    if (!lenient) return GMO_OUT_OF_BOUNDS;
    xmin = clampd(xmin, -180.0, 180.0); ymin = clampd(ymin, -90.0, 90.0); zmin = clampd(zmin, 0.0, zhi);
    xmax = clampd(xmax, -180.0, 180.0); ymax = clampd(ymax, -90.0, 90.0); zmax = clampd(zmax, 0.0, zhi);
  }
  const double zsize = zhi - 0.0;
  n[0] = (xmin - -180.0) / 360.0; n[1] = (ymin - -90.0) / 180.0; n[2] = (zmin - 0.0) / zsize;
  n[3] = (xmax - -180.0) / 360.0; n[4] = (ymax - -90.0) / 180.0; n[5] = (zmax - 0.0) / zsize;
  return GMO_OK;
}

/* XZ3SFC.index (XZ3SFC.scala:53-76) */
int gmo_xz3_index(int g, int period, double xmin, double ymin, double zmin, double xmax, double ymax,
                  double zmax, int lenient, int64_t* out) {
  double n[6];
  int st = xz3_normalize(period, xmin, ymin, zmin, xmax, ymax, zmax, lenient, n);
  if (st) { *out = 0; return st; }
  double maxdim = jmax(jmax(n[3] - n[0], n[4] - n[1]), n[5] - n[2]);
  double mins[3] = {n[0], n[1], n[2]}, maxs[3] = {n[3], n[4], n[5]};
  int length = xz_length(g, maxdim, mins, maxs, 3);
  *out = xz3_seqcode(g, n[0], n[1], n[2], length);
  return GMO_OK;
}

/* column batches of XZ2SFC.index / XZ3SFC.index (the bench's strided full-size parity samples) */
void gmo_xz2_index_batch(int g, const double* xmin, const double* ymin, const double* xmax, const double* ymax,
                         int64_t n, int lenient, int64_t* out, uint8_t* status) {
  for (int64_t i = 0; i < n; i++) {
    const int st = gmo_xz2_index(g, xmin[i], ymin[i], xmax[i], ymax[i], lenient, &out[i]);
    if (status) status[i] = (uint8_t)st;
  }
}
void gmo_xz3_index_batch(int g, int period, const double* xmin, const double* ymin, const double* zmin,
                         const double* xmax, const double* ymax, const double* zmax, int64_t n, int lenient,
                         int64_t* out, uint8_t* status) {
  for (int64_t i = 0; i < n; i++) {
    const int st = gmo_xz3_index(g, period, xmin[i], ymin[i], zmin[i], xmax[i], ymax[i], zmax[i], lenient, &out[i]);
    if (status) status[i] = (uint8_t)st;
  }
}

typedef struct { double mn[3], mx[3], len; int term; } xel;
typedef struct { xel* v; int64_t head, tail, cap; } xqueue;
static void xq_push(xqueue* q, const xel* e) {
  if (q->tail == q->cap) {
    if (q->head > 0 && q->head >= q->cap / 2) {
      memmove(q->v, q->v + q->head, (size_t)(q->tail - q->head) * sizeof(xel)); q->tail -= q->head; q->head = 0;
    } else { q->cap = q->cap ? q->cap * 2 : 256; q->v = (xel*)realloc(q->v, (size_t)q->cap * sizeof(xel)); }
  }
  q->v[q->tail++] = *e;
}

/* XElement.children (XZ2SFC.scala:406-415, XZ3SFC.scala:449-463): child c has bit0 = x upper half,
   bit1 = y upper half, bit2 = z upper half, in that enumeration order */
static void xel_children(int dims, const xel* p, xqueue* q) {
  double c[3];
  for (int d = 0; d < dims; d++) c[d] = (p->mn[d] + p->mx[d]) / 2.0;
  double len = p->len / 2.0;
  for (int k = 0; k < (1 << dims); k++) {
    xel e = *p; e.len = len; e.term = 0;
    for (int d = 0; d < dims; d++) {
      if (k >> d & 1) e.mn[d] = c[d]; else e.mx[d] = c[d];
    }
    xq_push(q, &e);
  }
}

/* XZ ranges BFS (XZ2SFC.scala:146-252, XZ3SFC.scala:156-262). q = normalized windows */
static int64_t xz_ranges_norm(int dims, int g, const double* win, int nq, int64_t range_stop,
                              gmo_range* out, int64_t cap) {
  rvec ranges = {0};
  xqueue q = {0};
  int quads = 1 << dims;
  const int64_t base = dims == 2 ? 4 : 8, div = dims == 2 ? 3 : 7;
  xel root; root.term = 0; root.len = 1.0;
  for (int d = 0; d < 3; d++) { root.mn[d] = 0.0; root.mx[d] = 1.0; }
  xel_children(dims, &root, &q);          /* LevelOneElements */
  xel term; memset(&term, 0, sizeof term); term.term = 1;
  xq_push(&q, &term);
  int level = 1;
  (void)quads;
#define XSEQ(e, lvl) (dims == 2 ? xz2_seqcode(g, (e)->mn[0], (e)->mn[1], (lvl)) \
                                : xz3_seqcode(g, (e)->mn[0], (e)->mn[1], (e)->mn[2], (lvl)))
  while (level < g && (q.tail - q.head) > 0 && ranges.n < range_stop) {
    xel next = q.v[q.head++];
    if (next.term) {
      if ((q.tail - q.head) > 0) { level += 1; xq_push(&q, &term); }
    } else {
      g_nodes_checked++;
      int contained = 0, overlapped = 0;
      for (int i = 0; i < nq && !contained; i++) {
        const double* w = win + 2 * dims * i;  /* mins then maxs */
        int c = 1;
        for (int d = 0; d < dims; d++) c = c && (w[d] <= next.mn[d]);
        for (int d = 0; d < dims; d++) c = c && (w[dims + d] >= next.mx[d] + next.len);
        contained = c;
      }
      if (!contained) {
        for (int i = 0; i < nq && !overlapped; i++) {
          const double* w = win + 2 * dims * i;
          int o = 1;
          for (int d = 0; d < dims; d++) o = o && (w[dims + d] >= next.mn[d]);
          for (int d = 0; d < dims; d++) o = o && (w[d] <= next.mx[d] + next.len);
          overlapped = o;
        }
      }
      if (contained) {
        int64_t mn = XSEQ(&next, level);
        rvec_push(&ranges, mn, mn + (ipow(base, g - level + 1) - 1) / div, 1);
      } else if (overlapped) {
        int64_t mn = XSEQ(&next, level);
        rvec_push(&ranges, mn, mn, 0);
        xel_children(dims, &next, &q);
      }
    }
  }
  while ((q.tail - q.head) > 0) {
    xel e = q.v[q.head++];
    if (e.term) level += 1;
    else {
      int64_t mn = XSEQ(&e, level);
      rvec_push(&ranges, mn, mn + (ipow(base, g - level + 1) - 1) / div, 0);
    }
  }
#undef XSEQ
  free(q.v);
  int64_t m = sort_merge(&ranges, out, cap);
  free(ranges.v);
  return m;
}

/* XZ2SFC.ranges(queries, maxRanges) (XZ2SFC.scala:130-137): q = nq*(xmin,ymin,xmax,ymax) */
int64_t gmo_xz2_ranges(int g, const double* q, int nq, int max_ranges, gmo_range* out, int64_t cap) {
  double* w = (double*)malloc(sizeof(double) * 4 * (size_t)(nq > 0 ? nq : 1));
  for (int i = 0; i < nq; i++) {
    double n[4];
    int st = xz2_normalize(q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3], 0, n);
    if (st) { free(w); return INT64_MIN + st; }
    w[4 * i] = n[0]; w[4 * i + 1] = n[1]; w[4 * i + 2] = n[2]; w[4 * i + 3] = n[3];
  }
  int64_t r = xz_ranges_norm(2, g, w, nq, max_ranges, out, cap);
  free(w);
  return r;
}

/* XZ3SFC.ranges (XZ3SFC.scala:139-147): q = nq*(xmin,ymin,zmin,xmax,ymax,zmax) */
int64_t gmo_xz3_ranges(int g, int period, const double* q, int nq, int max_ranges, gmo_range* out, int64_t cap) {
  double* w = (double*)malloc(sizeof(double) * 6 * (size_t)(nq > 0 ? nq : 1));
  for (int i = 0; i < nq; i++) {
    double n[6];
    const double* a = q + 6 * i;
    int st = xz3_normalize(period, a[0], a[1], a[2], a[3], a[4], a[5], 0, n);
    if (st) { free(w); return INT64_MIN + st; }
    for (int k = 0; k < 6; k++) w[6 * i + k] = n[k];
  }
  int64_t r = xz_ranges_norm(3, g, w, nq, max_ranges, out, cap);
  free(w);
  return r;
}

/* ------------------------------------------------------------------ */
/* Z3Filter / Z2Filter (idx/filters/Z3Filter.scala, Z2Filter.scala)    */
/* ------------------------------------------------------------------ */

static int32_t be_i32(const uint8_t* p) { return (int32_t)((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]); }
static int16_t be_i16(const uint8_t* p) { return (int16_t)(uint16_t)((uint16_t)p[0] << 8 | p[1]); }
static int64_t be_i64(const uint8_t* p) { uint64_t v = 0; for (int i = 0; i < 8; i++) v = v << 8 | p[i]; return (int64_t)v; }

typedef struct {
  int32_t nxy; const uint8_t* xy;   /* nxy * 4 BE ints */
  int32_t nt; const uint8_t** t; int32_t* tlen;  /* per epoch pointer to 2*len ints, NULL for null */
  int16_t min_epoch, max_epoch;
} z3f;

/* Z3Filter.deserializeFromBytes (Z3Filter.scala:139-153) */
static int z3f_parse(const uint8_t* b, size_t len, z3f* f) {
  size_t o = 0;
  if (len < 4) return -1;
  f->nxy = be_i32(b); o = 4;
  if (f->nxy < 0 || o + (size_t)f->nxy * 16 > len) return -1;
  f->xy = b + o; o += (size_t)f->nxy * 16;
  if (o + 4 > len) return -1;
  f->nt = be_i32(b + o); o += 4;
  if (f->nt < 0) return -1;
  f->t = (const uint8_t**)calloc((size_t)f->nt + 1, sizeof(uint8_t*));
  f->tlen = (int32_t*)calloc((size_t)f->nt + 1, sizeof(int32_t));
  for (int i = 0; i < f->nt; i++) {
    if (o + 4 > len) return -1;
    int32_t l = be_i32(b + o); o += 4;
    if (l == -1) { f->t[i] = NULL; f->tlen[i] = 0; }
    else { if (l < 0 || o + (size_t)l * 8 > len) return -1; f->t[i] = b + o; f->tlen[i] = l; o += (size_t)l * 8; }
  }
  if (o + 4 > len) return -1;
  f->min_epoch = be_i16(b + o); f->max_epoch = be_i16(b + o + 2);
  return 0;
}
static void z3f_free(z3f* f) { free(f->t); free(f->tlen); }

/* Z3Filter.inBounds / pointInBounds / timeInBounds (Z3Filter.scala:26-62) */
static int z3f_in_bounds(const z3f* f, int16_t epoch, int64_t z) {
  int32_t x = gmo_z3_combine(z), y = gmo_z3_combine(z >> 1);
  int pin = 0;
  for (int i = 0; i < f->nxy; i++) {
    const uint8_t* q = f->xy + 16 * i;
    if (x >= be_i32(q) && x <= be_i32(q + 8) && y >= be_i32(q + 4) && y <= be_i32(q + 12)) { pin = 1; break; }
  }
  if (!pin) return 0;
  if (epoch > f->max_epoch || epoch < f->min_epoch) return 1;
  int idx = epoch - f->min_epoch;
  if (idx >= f->nt || f->t[idx] == NULL) return 1;  /* Java would throw AIOOBE past nt; never built that way */
  int32_t t = gmo_z3_combine(z >> 2);
  for (int i = 0; i < f->tlen[idx]; i++) {
    const uint8_t* q = f->t[idx] + 8 * i;
    if (t >= be_i32(q) && t <= be_i32(q + 4)) return 1;
  }
  return 0;
}

int gmo_z3filter_in_bounds(const uint8_t* filter, size_t len, const uint8_t* row, int offset) {
  z3f f; memset(&f, 0, sizeof f);
  if (z3f_parse(filter, len, &f)) { z3f_free(&f); return -1; }
  int r = z3f_in_bounds(&f, be_i16(row + offset), be_i64(row + offset + 2));
  z3f_free(&f);
  return r;
}

int64_t gmo_z3filter_scan(const uint8_t* filter, size_t len, const int16_t* bin_ranges, int n_bin_ranges,
                          const int16_t* bin, const int64_t* z, int64_t n, uint8_t* match) {
  z3f f; memset(&f, 0, sizeof f);
  if (z3f_parse(filter, len, &f)) { z3f_free(&f); return -1; }
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; i++) {
    int ok = n_bin_ranges <= 0;
    for (int r = 0; r < n_bin_ranges && !ok; r++) ok = bin[i] >= bin_ranges[2 * r] && bin[i] <= bin_ranges[2 * r + 1];
    ok = ok && z3f_in_bounds(&f, bin[i], z[i]);
    if (match) match[i] = (uint8_t)ok;
    cnt += ok;
  }
  z3f_free(&f);
  return cnt;
}

/* Z2Filter.inBounds (Z2Filter.scala:20-35) */
static int z2f_in_bounds(const uint8_t* b, int32_t nxy, int64_t z) {
  int32_t x = gmo_z2_combine(z), y = gmo_z2_combine(z >> 1);
  for (int i = 0; i < nxy; i++) {
    const uint8_t* q = b + 4 + 16 * i;
    if (x >= be_i32(q) && x <= be_i32(q + 8) && y >= be_i32(q + 4) && y <= be_i32(q + 12)) return 1;
  }
  return 0;
}
int gmo_z2filter_in_bounds(const uint8_t* filter, size_t len, const uint8_t* row, int offset) {
  if (len < 4) return -1;
  int32_t nxy = be_i32(filter);
  if (nxy < 0 || 4 + (size_t)nxy * 16 > len) return -1;
  return z2f_in_bounds(filter, nxy, be_i64(row + offset));
}
int64_t gmo_z2filter_scan(const uint8_t* filter, size_t len, const int64_t* z, int64_t n, uint8_t* match) {
  if (len < 4) return -1;
  int32_t nxy = be_i32(filter);
  if (nxy < 0 || 4 + (size_t)nxy * 16 > len) return -1;
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; i++) { int ok = z2f_in_bounds(filter, nxy, z[i]); if (match) match[i] = (uint8_t)ok; cnt += ok; }
  return cnt;
}

/* strict filter: GeoTools BBOXImpl on a point (GeometryProcessing.scala:129; inclusive edges -- parity
   unpinned beyond AccumuloDataStoreQueryTest.scala:575-684) AND FastDuring
   (geomesa-filter/.../FastTemporalOperator.scala:123-126: date.after(beg) && date.before(end)) */
int64_t gmo_strict_scan(const double* x, const double* y, const int64_t* t_ms, int64_t n,
                        const double* bbox, int has_during, int64_t lo, int64_t hi, uint8_t* match) {
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; i++) {
    int ok = x[i] >= bbox[0] && x[i] <= bbox[2] && y[i] >= bbox[1] && y[i] <= bbox[3];
    if (has_during) ok = ok && t_ms[i] > lo && t_ms[i] < hi;
    if (match) match[i] = (uint8_t)ok;
    cnt += ok;
  }
  return cnt;
}

/* ------------------------------------------------------------------ */
/* JTS 1.20.0 semantics for Geometry.contains(point)                   */
/* (third-party, not vendored; call site geomesa-spark-jts/.../         */
/*  SpatialRelationFunctions.scala:29)                                  */
/* ------------------------------------------------------------------ */

typedef struct { double hi, lo; } dd;
static const double DD_SPLIT = 134217729.0; /* 2^27+1 */

/* DD.selfAdd(double) */
static dd dd_add_d(dd a, double y) {
  double H, h, S, s, e, f;
  S = a.hi + y; e = S - a.hi; s = S - e; s = (y - e) + (a.hi - s);
  f = s + a.lo; H = S + f; h = f + (S - H);
  dd r; r.hi = H + h; r.lo = h + (H - r.hi); return r;
}
/* DD.selfAdd(hi, lo) */
static dd dd_add(dd a, double yhi, double ylo) {
  double H, h, T, t, S, s, e, f;
  S = a.hi + yhi; T = a.lo + ylo; e = S - a.hi; f = T - a.lo;
  s = S - e; t = T - f; s = (yhi - e) + (a.hi - s); t = (ylo - f) + (a.lo - t);
  e = s + T; H = S + e; h = e + (S - H); e = t + h;
  dd r; r.hi = H + e; r.lo = e + (H - r.hi); return r;
}
/* DD.selfMultiply(hi, lo) */
static dd dd_mul(dd a, double yhi, double ylo) {
  double hx, tx, hy, ty, C, c;
  C = DD_SPLIT * a.hi; hx = C - a.hi; c = DD_SPLIT * yhi;
  hx = C - hx; tx = a.hi - hx; hy = c - yhi;
  C = a.hi * yhi; hy = c - hy; ty = yhi - hy;
  c = ((((hx * hy - C) + hx * ty) + tx * hy) + tx * ty) + (a.hi * ylo + a.lo * yhi);
  double zhi = C + c; hx = C - zhi; double zlo = c + hx;
  dd r; r.hi = zhi; r.lo = zlo; return r;
}
static int dd_signum(dd a) { if (a.hi > 0) return 1; if (a.hi < 0) return -1; if (a.lo > 0) return 1; if (a.lo < 0) return -1; return 0; }
static int sgn(double x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

/* CGAlgorithmsDD.orientationIndexFilter + orientationIndex */
int gmo_orientation_index(double p1x, double p1y, double p2x, double p2y, double qx, double qy) {
  double detleft = (p1x - qx) * (p2y - qy);
  double detright = (p1y - qy) * (p2x - qx);
  double det = detleft - detright, detsum;
  int filt;
  if (detleft > 0.0) {
    if (detright <= 0.0) return sgn(det);
    detsum = detleft + detright;
  } else if (detleft < 0.0) {
    if (detright >= 0.0) return sgn(det);
    detsum = -detleft - detright;
  } else {
    return sgn(det);
  }
  double errbound = 1e-15 * detsum;
  if ((det >= errbound) || (-det >= errbound)) return sgn(det);
  filt = 2; (void)filt;
  dd dx1 = {p2x, 0.0}; dx1 = dd_add_d(dx1, -p1x);
  dd dy1 = {p2y, 0.0}; dy1 = dd_add_d(dy1, -p1y);
  dd dx2 = {qx, 0.0};  dx2 = dd_add_d(dx2, -p2x);
  dd dy2 = {qy, 0.0};  dy2 = dd_add_d(dy2, -p2y);
  dd a = dd_mul(dx1, dy2.hi, dy2.lo);
  dd b = dd_mul(dy1, dx2.hi, dx2.lo);
  dd r = dd_add(a, -b.hi, -b.lo);
  return dd_signum(r);
}

#define LOC_EXTERIOR 0
#define LOC_BOUNDARY 1
#define LOC_INTERIOR 2

/* RayCrossingCounter.locatePointInRing / countSegment */
static int locate_in_ring(double px, double py, const double* vx, const double* vy, int n) {
  /* PointLocator.locateInPolygonRing: ring envelope check first */
  double mnx = vx[0], mxx = vx[0], mny = vy[0], mxy = vy[0];
  for (int i = 1; i < n; i++) {
    if (vx[i] < mnx) mnx = vx[i]; if (vx[i] > mxx) mxx = vx[i];
    if (vy[i] < mny) mny = vy[i]; if (vy[i] > mxy) mxy = vy[i];
  }
  if (!(px >= mnx && px <= mxx && py >= mny && py <= mxy)) return LOC_EXTERIOR;
  int crossings = 0;
  for (int i = 1; i < n; i++) {
    double p1x = vx[i], p1y = vy[i], p2x = vx[i - 1], p2y = vy[i - 1];
    if (p1x < px && p2x < px) continue;
    if (px == p2x && py == p2y) return LOC_BOUNDARY;
    if (p1y == py && p2y == py) {
      double minx = p1x, maxx = p2x;
      if (minx > maxx) { minx = p2x; maxx = p1x; }
      if (px >= minx && px <= maxx) return LOC_BOUNDARY;
      continue;
    }
    if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
      int orient = gmo_orientation_index(p1x, p1y, p2x, p2y, px, py);
      if (orient == 0) return LOC_BOUNDARY;
      if (p2y < p1y) orient = -orient;
      if (orient == 1) crossings++;
    }
  }
  return (crossings % 2) == 1 ? LOC_INTERIOR : LOC_EXTERIOR;
}

/* PointLocator.locateInPolygon */
static int locate_in_polygon(const gmo_polyset* ps, int part, double px, double py) {
  int r0 = ps->part_ring_off[part], r1 = ps->part_ring_off[part + 1];
  if (r1 <= r0) return LOC_EXTERIOR;
  int v0 = ps->ring_vert_off[r0], v1 = ps->ring_vert_off[r0 + 1];
  if (v1 - v0 < 1) return LOC_EXTERIOR;
  int shell = locate_in_ring(px, py, ps->vx + v0, ps->vy + v0, v1 - v0);
  if (shell != LOC_INTERIOR) return shell;
  for (int r = r0 + 1; r < r1; r++) {
    int h0 = ps->ring_vert_off[r], h1 = ps->ring_vert_off[r + 1];
    if (h1 - h0 < 1) continue;
    int hl = locate_in_ring(px, py, ps->vx + h0, ps->vy + h0, h1 - h0);
    if (hl == LOC_INTERIOR) return LOC_EXTERIOR;
    if (hl == LOC_BOUNDARY) return LOC_BOUNDARY;
  }
  return LOC_INTERIOR;
}

/* PointLocator.locate with the Mod-2 boundary rule over the polygon components */
int gmo_locate(const gmo_polyset* ps, int poly, double px, double py) {
  int p0 = ps->poly_part_off[poly], p1 = ps->poly_part_off[poly + 1];
  int is_in = 0, nb = 0;
  for (int p = p0; p < p1; p++) {
    int l = locate_in_polygon(ps, p, px, py);
    if (l == LOC_INTERIOR) is_in = 1;
    if (l == LOC_BOUNDARY) nb++;
  }
  if (nb % 2 == 1) return LOC_BOUNDARY;
  if (nb > 0 || is_in) return LOC_INTERIOR;
  return LOC_EXTERIOR;
}

static void poly_env(const gmo_polyset* ps, int poly, double* e) {
  e[0] = INFINITY; e[1] = INFINITY; e[2] = -INFINITY; e[3] = -INFINITY;
  int p0 = ps->poly_part_off[poly], p1 = ps->poly_part_off[poly + 1];
  for (int p = p0; p < p1; p++) {
    int r0 = ps->part_ring_off[p];
    if (ps->part_ring_off[p + 1] <= r0) continue;
    for (int v = ps->ring_vert_off[r0]; v < ps->ring_vert_off[r0 + 1]; v++) {
      if (ps->vx[v] < e[0]) e[0] = ps->vx[v]; if (ps->vx[v] > e[2]) e[2] = ps->vx[v];
      if (ps->vy[v] < e[1]) e[1] = ps->vy[v]; if (ps->vy[v] > e[3]) e[3] = ps->vy[v];
    }
  }
}

/* Geometry.contains(point): envelope covers, then relate -> interior (RectangleContains gives the
   same strict-interior answer for rectangles). Empty geometry -> false. */
int gmo_contains(const gmo_polyset* ps, int poly, double px, double py) {
  double e[4]; poly_env(ps, poly, e);
  if (!(px >= e[0] && px <= e[2] && py >= e[1] && py <= e[3])) return 0;
  return gmo_locate(ps, poly, px, py) == LOC_INTERIOR;
}

/* Geometry.intersects(point): envelopes intersect, then relate -> not exterior
   (RectangleIntersects, JTS 1.20, gives the same closed-rectangle answer for a point). */
int gmo_intersects(const gmo_polyset* ps, int poly, double px, double py) {
  double e[4]; poly_env(ps, poly, e);
  if (!(px >= e[0] && px <= e[2] && py >= e[1] && py <= e[3])) return 0;
  return gmo_locate(ps, poly, px, py) != LOC_EXTERIOR;
}

/* Full filter of a point query (Z3IndexKeySpace useFullFilter, Z3IndexKeySpace.scala:240-254):
   BBOX (inclusive) AND during (exclusive, ms) AND the OR over the query geometries of
   INTERSECTS(geom, P) (op 1) or CONTAINS(P, geom) / WITHIN(geom, P) (op 2)
   (GeometryProcessing.process splits a query geometry into an OR of parts, GeometryProcessing.scala:104-136).
   bbox NULL = no BBOX term; ps NULL or op 0 = no geometry term. */
int64_t gmo_query_scan(const double* x, const double* y, const int64_t* t_ms, int64_t n, const double* bbox,
                       int has_during, int64_t lo, int64_t hi, const gmo_polyset* ps, int op, uint8_t* match) {
  int64_t cnt = 0;
  for (int64_t i = 0; i < n; i++) {
    int ok = 1;
    if (bbox) ok = x[i] >= bbox[0] && x[i] <= bbox[2] && y[i] >= bbox[1] && y[i] <= bbox[3];
    if (ok && has_during) ok = t_ms[i] > lo && t_ms[i] < hi;
    if (ok && ps && op) {
      int any = 0;
      for (int k = 0; k < ps->n_polys && !any; k++)
        any = op == 1 ? gmo_intersects(ps, k, x[i], y[i]) : gmo_contains(ps, k, x[i], y[i]);
      ok = any;
    }
    if (match) match[i] = (uint8_t)ok;
    cnt += ok;
  }
  return cnt;
}

/* ---- join: uniform grid over polygon envelopes (the restatement of RelationUtils.grid +
   GeoMesaJoinRelation.sweeplineJoin candidate generation), then JTS contains per candidate ---- */
typedef struct {
  const gmo_polyset* ps; double* env; int gx, gy; double minx, miny, maxx, maxy, cw, ch;
  int32_t* cell_off; int32_t* cell_poly;
  const double* px; const double* py; int64_t lo, hi;
  int64_t* pt; int32_t* pl; int64_t n, cap;
  int op;                 /* 2 = contains (interior), 1 = intersects (interior or boundary) */
  const int64_t* pedges;  /* edges per polygon, for the candidate-edge count E_c */
  int64_t cand_edges;
} join_task;

static inline int cell_of(double v, double mn, double w, int g) {
  double c = floor((v - mn) / w);
  if (!(c >= 0)) return 0;
  if (c >= g) return g - 1;
  return (int)c;
}

static void* join_worker(void* arg) {
  join_task* t = (join_task*)arg;
  for (int64_t i = t->lo; i < t->hi; i++) {
    double x = t->px[i], y = t->py[i];
    if (!(x >= t->minx && x <= t->maxx && y >= t->miny && y <= t->maxy)) continue;
    int cx = cell_of(x, t->minx, t->cw, t->gx), cy = cell_of(y, t->miny, t->ch, t->gy);
    int c = cy * t->gx + cx;
    for (int k = t->cell_off[c]; k < t->cell_off[c + 1]; k++) {
      int p = t->cell_poly[k];
      const double* e = t->env + 4 * p;
      if (!(x >= e[0] && x <= e[2] && y >= e[1] && y <= e[3])) continue;
      t->cand_edges += t->pedges[p];
      const int loc = gmo_locate(t->ps, p, x, y);
      if (t->op == 1 ? loc == LOC_EXTERIOR : loc != LOC_INTERIOR) continue;
      if (t->n == t->cap) { t->cap = t->cap ? t->cap * 2 : 1024; t->pt = (int64_t*)realloc(t->pt, 8 * (size_t)t->cap); t->pl = (int32_t*)realloc(t->pl, 4 * (size_t)t->cap); }
      t->pt[t->n] = i; t->pl[t->n] = p; t->n++;
    }
  }
  return NULL;
}

static int cmp_i32(const void* a, const void* b) { int32_t x = *(const int32_t*)a, y = *(const int32_t*)b; return (x > y) - (x < y); }

int64_t gmo_pip_join(const gmo_polyset* ps, const double* px, const double* py, int64_t n,
                     int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int nthreads) {
  return gmo_pip_join_ex(ps, px, py, n, pt_ids, poly_ids, cap, nthreads, 2, NULL);
}

/* The join with the condition's predicate (op 2 = ST_Contains, 1 = ST_Intersects,
   SpatialRelationFunctions.scala:29-34); *cand_edges (optional) receives E_c = the edges of every
   (point, polygon) pair whose envelope test passed, i.e. the orientation tests a JTS RayCrossingCounter
   walk makes over the candidates (the FP64 work of SURVEY 8(d)). */
int64_t gmo_pip_join_ex(const gmo_polyset* ps, const double* px, const double* py, int64_t n,
                        int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int nthreads, int op, int64_t* cand_edges) {
  int np = ps->n_polys;
  if (cand_edges) *cand_edges = 0;
  if (np <= 0 || n <= 0) return 0;
  int64_t* pedges = (int64_t*)calloc((size_t)np, sizeof(int64_t));
  for (int p = 0; p < np; p++)
    for (int q = ps->poly_part_off[p]; q < ps->poly_part_off[p + 1]; q++)
      for (int r = ps->part_ring_off[q]; r < ps->part_ring_off[q + 1]; r++) {
        const int nv = ps->ring_vert_off[r + 1] - ps->ring_vert_off[r];
        pedges[p] += nv > 1 ? nv - 1 : 0;
      }
  double* env = (double*)malloc(sizeof(double) * 4 * (size_t)np);
  double g[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
  for (int p = 0; p < np; p++) {
    poly_env(ps, p, env + 4 * p);
    if (env[4 * p] > env[4 * p + 2]) continue; /* empty */
    if (env[4 * p] < g[0]) g[0] = env[4 * p]; if (env[4 * p + 1] < g[1]) g[1] = env[4 * p + 1];
    if (env[4 * p + 2] > g[2]) g[2] = env[4 * p + 2]; if (env[4 * p + 3] > g[3]) g[3] = env[4 * p + 3];
  }
  if (!(g[0] <= g[2])) { free(env); free(pedges); return 0; }
  int gx = 1, gy = 1;
  while (gx * gy < 4 * np && gx < 1024) { gx *= 2; gy *= 2; }
  double cw = (g[2] - g[0]) / gx, ch = (g[3] - g[1]) / gy;
  if (!(cw > 0)) cw = 1.0; if (!(ch > 0)) ch = 1.0;
  int ncell = gx * gy;
  int32_t* cnt = (int32_t*)calloc((size_t)ncell + 1, sizeof(int32_t));
  for (int p = 0; p < np; p++) {
    if (env[4 * p] > env[4 * p + 2]) continue;
    int x0 = cell_of(env[4 * p], g[0], cw, gx), x1 = cell_of(env[4 * p + 2], g[0], cw, gx);
    int y0 = cell_of(env[4 * p + 1], g[1], ch, gy), y1 = cell_of(env[4 * p + 3], g[1], ch, gy);
    for (int cy = y0; cy <= y1; cy++) for (int cx = x0; cx <= x1; cx++) cnt[cy * gx + cx + 1]++;
  }
  for (int c = 0; c < ncell; c++) cnt[c + 1] += cnt[c];
  int32_t* fill = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
  memcpy(fill, cnt, sizeof(int32_t) * (size_t)ncell);
  int32_t* cell_poly = (int32_t*)malloc(sizeof(int32_t) * (size_t)(cnt[ncell] > 0 ? cnt[ncell] : 1));
  for (int p = 0; p < np; p++) {
    if (env[4 * p] > env[4 * p + 2]) continue;
    int x0 = cell_of(env[4 * p], g[0], cw, gx), x1 = cell_of(env[4 * p + 2], g[0], cw, gx);
    int y0 = cell_of(env[4 * p + 1], g[1], ch, gy), y1 = cell_of(env[4 * p + 3], g[1], ch, gy);
    for (int cy = y0; cy <= y1; cy++) for (int cx = x0; cx <= x1; cx++) cell_poly[fill[cy * gx + cx]++] = p;
  }
  for (int c = 0; c < ncell; c++) qsort(cell_poly + cnt[c], (size_t)(cnt[c + 1] - cnt[c]), sizeof(int32_t), cmp_i32);
  if (nthreads < 1) nthreads = 1;
  join_task* tasks = (join_task*)calloc((size_t)nthreads, sizeof(join_task));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  int64_t chunk = (n + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; k++) {
    join_task* t = &tasks[k];
    t->ps = ps; t->env = env; t->gx = gx; t->gy = gy; t->minx = g[0]; t->miny = g[1]; t->maxx = g[2]; t->maxy = g[3]; t->cw = cw; t->ch = ch;
    t->cell_off = cnt; t->cell_poly = cell_poly; t->px = px; t->py = py; t->op = op; t->pedges = pedges;
    t->lo = (int64_t)k * chunk; t->hi = t->lo + chunk < n ? t->lo + chunk : n; if (t->lo > n) t->lo = n;
    if (nthreads == 1) join_worker(t); else pthread_create(&th[k], NULL, join_worker, t);
  }
  int64_t total = 0;
  for (int k = 0; k < nthreads; k++) { if (nthreads > 1) pthread_join(th[k], NULL); }
  for (int k = 0; k < nthreads; k++) {
    join_task* t = &tasks[k];
    for (int64_t j = 0; j < t->n; j++) {
      if (total + j < cap) { pt_ids[total + j] = t->pt[j]; poly_ids[total + j] = t->pl[j]; }
    }
    total += t->n;
    if (cand_edges) *cand_edges += t->cand_edges;
    free(t->pt); free(t->pl);
  }
  free(tasks); free(th); free(cell_poly); free(fill); free(cnt); free(env); free(pedges);
  return total <= cap ? total : -total;
}

/* ---- batch of the range decompositions (the bench's CPU baseline and its full-size parity): nq
   single-box queries on nthreads pthreads; totals of merged ranges and nodes checked, and optionally
   each query's merged-range count (counts[nq]) and, given offsets[nq] from those counts, the ranges
   themselves at out + offsets[i] */
typedef struct {
  int kind, period, g, max_ranges, pad;  /* kind 3 = Z3, 12 = XZ2, 13 = XZ3 */
  const double* q; const int64_t* t;
  int64_t lo, hi, ranges, nodes;
  int64_t* counts; const int64_t* offsets; gmo_range* out;
} rbatch_task;

static void* rbatch_worker(void* arg) {
  rbatch_task* k = (rbatch_task*)arg;
  int64_t cap = 1 << 16;
  gmo_range* out = (gmo_range*)malloc(sizeof(gmo_range) * (size_t)cap);
  g_nodes_checked = 0;
  int64_t nodes = 0;
  for (int64_t i = k->lo; i < k->hi; i++) {
    int64_t m;
    for (;;) {
      g_nodes_checked = 0;
      if (k->kind == 3) m = gmo_z3_ranges(k->period, 21, k->q + 4 * i, 1, k->t + 2 * i, 1, 64, k->max_ranges, out, cap);
      else if (k->kind == 12) m = gmo_xz2_ranges(k->g, k->q + 4 * i, 1, k->max_ranges, out, cap);
      else m = gmo_xz3_ranges(k->g, k->period, k->q + 6 * i, 1, k->max_ranges, out, cap);
      if (m < 0 && m > -(INT64_C(1) << 62)) {   /* capacity: grow and redo this query */
        cap = -m;
        out = (gmo_range*)realloc(out, sizeof(gmo_range) * (size_t)cap);
        continue;
      }
      break;
    }
    nodes += g_nodes_checked;
    if (m > 0) k->ranges += m;
    if (k->counts) k->counts[i] = m;
    if (k->out && k->offsets && m > 0) memcpy(k->out + k->offsets[i], out, sizeof(gmo_range) * (size_t)m);
  }
  k->nodes = nodes;
  free(out);
  return NULL;
}

int gmo_ranges_batch(int kind, int period, int g, const double* q, const int64_t* t, int64_t nq, int max_ranges,
                     int nthreads, int64_t* total_ranges, int64_t* total_nodes, int64_t* counts,
                     const int64_t* offsets, gmo_range* out) {
  if (nthreads < 1) nthreads = 1;
  rbatch_task* tasks = (rbatch_task*)calloc((size_t)nthreads, sizeof(rbatch_task));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  const int64_t chunk = (nq + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; k++) {
    rbatch_task* x = &tasks[k];
    x->kind = kind; x->period = period; x->g = g; x->max_ranges = max_ranges; x->q = q; x->t = t;
    x->counts = counts; x->offsets = offsets; x->out = out;
    x->lo = (int64_t)k * chunk; x->hi = x->lo + chunk < nq ? x->lo + chunk : nq;
    if (x->lo > nq) x->lo = nq;
    pthread_create(&th[k], NULL, rbatch_worker, x);
  }
  int64_t r = 0, nd = 0;
  for (int k = 0; k < nthreads; k++) { pthread_join(th[k], NULL); r += tasks[k].ranges; nd += tasks[k].nodes; }
  if (total_ranges) *total_ranges = r;
  if (total_nodes) *total_nodes = nd;
  free(tasks); free(th);
  return 0;
}
