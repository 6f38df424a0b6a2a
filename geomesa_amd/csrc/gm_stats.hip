// gm_stats.hip -- Z3Histogram.observe / unobserve over a batch of point features on gfx950.
//
// Reference: Z3Histogram (utils/stats/Z3Histogram.scala:101-128): per feature toKey (:80-86) =
// BinnedTime.timeToBinnedTime(period) + Z3SFC(period).index(centroid, offset, lenient), then
// binMap(timeBin).add(z, +-1) where the bin array is BinnedArray(LongBinning(length, (minZ, maxZ)))
// (utils/stats/BinnedArray.scala:59-64, 185-201) with minZ / maxZ the z of MinMaxGeometry.min / max
// (MinMax.scala:191-192) at sfc.time.min / max (Z3Histogram.scala:53-54).
//
// Shape: the same streaming read as the Z3 key kernel (24 B/point, 16-B pair loads) with the
// write side replaced by an increment.  Every workgroup keeps a private int32 copy of a block of
// time-bin rows of the [n_bins][length] counters in LDS (<= 32768 int32 = 128 KB) and flushes the
// nonzero counters with one 64-bit device atomic each at the end, so HBM traffic is the 24 B/point
// read plus grid x counters x 8 B; the grid is one resident wave of workgroups (1-2 per CU).  A
// histogram larger than one LDS block of int32 counters keeps three 21-bit counters per 64-bit word
// instead (WIDE below: 1024 x 54 week bins fit one pass), and beyond that takes up to
// HIST_MAX_PASSES passes over the points, one per row block; beyond that it adds straight into the
// 64-bit device counters (scattered per-lane device atomics run ~22 G/s on MI355X, so they only win
// over many passes).
#include <cmath>

#include "gm_keys.hpp"

namespace gm {

constexpr int HTPB = 1024;
constexpr int HIST_LDS_MAX = 32768;  // int32 counters per workgroup (128 KB of the 160 KB LDS)
// LDS for the WIDE counters, the row flags and what rounding leaves: 160 KB less the 8 KB spread table
// and the kernel's two scalars
constexpr int HIST_WIDE_BYTES = 163840 - 8192 - 64;
constexpr int HIST_MAX_PASSES = 4;

struct HistArgs {
  int64_t n;
  int length, bin_lo, n_bins;
  int64_t zmin, zmax;
  double bsize;  // LongBinning.binSize = (max - min).toDouble / length
  double inv_bsize;  // 1 / bsize when bsize is a power of two (x / 2^k == x * 2^-k exactly), else 0
  NDim lon, lat, tim;
  int row_lo, row_n;  // LDS pass: the time-bin rows [row_lo, row_lo + row_n) of the window it counts
  int tally;          // this launch reports skipped / outside features (the first pass only)
  int top_s, top_sh;  // TOP path (length 2^m, m <= 21): s = floor((63 - m) / 3), sh = 63 - m - 3 s
};

// LongBinning.directIndex (BinnedArray.scala:195-201); (value - min) is a Long, divided by a Double
__device__ __forceinline__ int long_bin_index(int64_t v, const HistArgs& a) {
  if (v < a.zmin || v > a.zmax) return -1;
  const double d = (double)(int64_t)((uint64_t)v - (uint64_t)a.zmin);
  const double q = floor(a.inv_bsize != 0.0 ? d * a.inv_bsize : d / a.bsize);
  const int i = q >= 2147483647.0 ? 2147483647 : (q <= -2147483648.0 ? (-2147483647 - 1) : (int)q);
  if (i < 0 || i > a.length) return -1;
  return i == a.length ? a.length - 1 : i;
}

// toKey + bin lookup for one feature; returns the flat counter index, -1 to drop, and classifies
// drops: *skip for a throwing toKey (the Scala code logs and moves on), *out for a time bin
// outside the caller's window [bin_lo, bin_lo + n_bins)
template <int PERIOD, bool UNOBS>
__device__ __forceinline__ int hist_slot(double x, double y, int64_t ms, const HistArgs& a, int& rb, int& skip,
                                         int& out) {
  int16_t b;
  int64_t off, z;
  uint8_t st = binned_time<PERIOD>(ms, b, off);
  if (st == ST_OK) st = z3_index_one<UNOBS>(x, y, off, a.lon, a.lat, a.tim, z);  // unobserve is lenient
  if (st != ST_OK) { ++skip; return -1; }
  rb = (int)b - a.bin_lo;
  if (rb < 0 || rb >= a.n_bins) { ++out; return -1; }
  const int i = long_bin_index(z, a);
  return i < 0 ? -1 : rb * a.length + i;
}

// hist_slot with the table spread; the bounds / lenient / normalize steps are z3_index_one's
template <int PERIOD, bool UNOBS>
__device__ __forceinline__ int hist_slot_tab(double x, double y, int64_t ms, const HistArgs& a, const uint32_t* sp,
                                             int& rb, int& skip, int& out) {
  int16_t b;
  int64_t off;
  if (binned_time<PERIOD>(ms, b, off) != ST_OK) { ++skip; return -1; }
  double td = (double)off;
  const bool inb = x >= a.lon.min && x <= a.lon.max && y >= a.lat.min && y <= a.lat.max && td >= a.tim.min &&
                   td <= a.tim.max;
  if (!inb) {
    if (!UNOBS) { ++skip; return -1; }
    x = x < a.lon.min ? a.lon.min : (x > a.lon.max ? a.lon.max : x);
    y = y < a.lat.min ? a.lat.min : (y > a.lat.max ? a.lat.max : y);
    td = td < a.tim.min ? a.tim.min : (td > a.tim.max ? a.tim.max : td);
  }
  const int64_t z = (int64_t)(z3_split_tab(normalize(a.lon, x), sp) | (z3_split_tab(normalize(a.lat, y), sp) << 1) |
                              (z3_split_tab(normalize(a.tim, td), sp) << 2));
  rb = (int)b - a.bin_lo;
  if (rb < 0 || rb >= a.n_bins) { ++out; return -1; }
  const int i = long_bin_index(z, a);
  return i < 0 ? -1 : rb * a.length + i;
}

// TOP path, length = 2^m (m <= 21).  The bin is floor(double(z) / 2^(63 - m)) (directIndex's Long ->
// Double conversion rounds z to 53 bits), i.e. the top m bits of z unless that rounding carries into
// them.  z interleaves the masked normalized dims (bit 3k + d = bit k of dim d), so z >> 3s is the
// interleave of the dims' bits >= s, and the top m bits are that >> sh: a few bits per dim instead of
// the 63-bit key.  A carry from the rounding (which starts below bit 11 of z) reaches bit 3s only
// through a run of ones, so when some dim has a zero among its bits [s - 4, s) -- a zero of z in
// [3s - 12, 3s) -- the top bits are the answer; otherwise (probability 2^-12) the exact full path
// below decides.
template <int PERIOD, bool UNOBS>
__device__ __forceinline__ int hist_slot_top(double x, double y, int64_t ms, const HistArgs& a, const uint32_t* sp,
                                             int& rb, int& skip, int& out) {
  int16_t b;
  int64_t off;
  if (binned_time<PERIOD>(ms, b, off) != ST_OK) { ++skip; return -1; }
  double td = (double)off;
  const bool inb = x >= a.lon.min && x <= a.lon.max && y >= a.lat.min && y <= a.lat.max && td >= a.tim.min &&
                   td <= a.tim.max;
  if (!inb) {
    if (!UNOBS) { ++skip; return -1; }
    x = x < a.lon.min ? a.lon.min : (x > a.lon.max ? a.lon.max : x);
    y = y < a.lat.min ? a.lat.min : (y > a.lat.max ? a.lat.max : y);
    td = td < a.tim.min ? a.tim.min : (td > a.tim.max ? a.tim.max : td);
  }
  rb = (int)b - a.bin_lo;
  if (rb < 0 || rb >= a.n_bins) { ++out; return -1; }
  const uint32_t xn = (uint32_t)normalize(a.lon, x) & 0x1fffffu, yn = (uint32_t)normalize(a.lat, y) & 0x1fffffu;
  const uint32_t tn = (uint32_t)normalize(a.tim, td) & 0x1fffffu;
  const int s = a.top_s;
  const uint32_t low = 15u << (s - 4);
  int i;
  if ((xn & yn & tn & low) != low) {
    i = (int)((spread3_11(xn >> s) | (spread3_11(yn >> s) << 1) | (spread3_11(tn >> s) << 2)) >> a.top_sh);
  } else {
    const int64_t z = (int64_t)(z3_split_tab((int32_t)xn, sp) | (z3_split_tab((int32_t)yn, sp) << 1) |
                                (z3_split_tab((int32_t)tn, sp) << 2));
    i = long_bin_index(z, a);
    if (i < 0) return -1;
  }
  return rb * a.length + i;
}

// WIDE: three 21-bit counters per 64-bit LDS word (55,296 counters -- 1024 x 54 week bins -- in one
// 144 KB pass, where int32 counters need 216 KB).  Increments are plain non-returning 64-bit LDS adds
// (ds_add_u64) of 1 << (21 k); a field cannot carry into its neighbour because the workgroup drains
// every field to the device counters (and resets it) before any field can have moved by 2^21 - 1
// (observe, fields from 0) or 2^20 - 1 (unobserve, fields biased at 2^20): the drain comes after a
// fixed number of block iterations, each of which counts at most HTPB * HU * 2 points.  So the hot loop
// carries no returning atomic and no per-point check (the former 16-bit halves took a returning LDS
// atomic per increment: 4.71-4.75 vs 4.36 ms per 1B points for int32 counters).  What the 1024 x 54
// histogram still pays over 512 x 54 int32 counters (4.72-4.76 vs 4.24-4.32 ms) is half the 64-bit
// adds (WIDE at 512: 4.47-4.51) and half the larger table; 32-bit adds for the two fields that lie
// inside one dword (fields 0 and 2) cost more (4.86-4.90: the lanes split over two LDS instructions),
// profiles/r5/hist_atomic_width_ab.txt.
constexpr int WBITS = 21;
constexpr uint64_t WMASK = (1ull << WBITS) - 1;
__device__ __forceinline__ uint64_t wide_bias(bool unobs) { return unobs ? (1ull << 20) : 0ull; }
__device__ __forceinline__ uint64_t wide_fill(bool unobs) {
  const uint64_t b = wide_bias(unobs);
  return b | (b << WBITS) | (b << (2 * WBITS));
}

template <bool SUB>
__device__ __forceinline__ void wide_add(uint64_t* wcnt, int c) {
  const int q = c / 3, k = c - 3 * q;
  if (SUB) atomicSub((unsigned long long*)&wcnt[q], 1ull << (WBITS * k));
  else atomicAdd((unsigned long long*)&wcnt[q], 1ull << (WBITS * k));
}

template <int PERIOD, bool UNOBS, bool VEC, bool WIDE, bool TOP>
__global__ __launch_bounds__(HTPB) void k_z3_hist_lds(const double* __restrict__ x, const double* __restrict__ y,
                                                      const int64_t* __restrict__ t, HistArgs a,
                                                      uint8_t* __restrict__ present,
                                                      unsigned long long* __restrict__ counts,
                                                      unsigned long long* __restrict__ tally) {
  extern __shared__ uint64_t lds64[];
  const int total = a.row_n * a.length;
  const int cw64 = WIDE ? (total + 2) / 3 : (total + 1) / 2;   // 64-bit words of counters
  int* cnt = (int*)lds64;                  // int32 counters [row_n * length] (!WIDE)
  uint64_t* wcnt = lds64;                  // 3 x 21-bit counters per word (WIDE)
  int* pres = (int*)(lds64 + cw64);        // [row_n]: bin present (observe sets, unobserve reads)
  uint32_t* sp = (uint32_t*)(pres + a.row_n);  // [2048]: spread3_11 table
  __shared__ int s_skip, s_out;
  counts += (int64_t)a.row_lo * a.length;
  present += a.row_lo;
  if (WIDE) for (int i = threadIdx.x; i < cw64; i += HTPB) wcnt[i] = wide_fill(UNOBS);
  else for (int i = threadIdx.x; i < total; i += HTPB) cnt[i] = 0;
  for (int i = threadIdx.x; i < a.row_n; i += HTPB) pres[i] = UNOBS ? (int)present[i] : 0;
  fill_spread_table(sp, threadIdx.x, HTPB);
  if (threadIdx.x == 0) { s_skip = 0; s_out = 0; }
  __syncthreads();
  int skip = 0, out = 0;
  auto one = [&](double xx, double yy, int64_t tt) {
    int rb = 0;
    int c = TOP ? hist_slot_top<PERIOD, UNOBS>(xx, yy, tt, a, sp, rb, skip, out)
                : hist_slot_tab<PERIOD, UNOBS>(xx, yy, tt, a, sp, rb, skip, out);
    rb -= a.row_lo;
    if (c < 0 || rb < 0 || rb >= a.row_n) return;
    c -= a.row_lo * a.length;
    if (UNOBS) {
      if (pres[rb]) {                        // binMap.get(timeBin).foreach(_.add(z, -1))
        if (WIDE) wide_add<true>(wcnt, c);
        else atomicAdd(&cnt[c], -1);
      }
    } else {
      // binMap.getOrElseUpdate(timeBin, newBins): a row is present iff one of its features was
      // counted; the drains and the flush derive it from the counters (no per-point LDS read)
      if (WIDE) wide_add<false>(wcnt, c);
      else atomicAdd(&cnt[c], 1);
    }
  };
  // every field's change since the last drain to the device counters (and, observing, the rows it
  // shows present); reset = the fields back to their bias.  All threads, two barriers.
  auto drain = [&](bool reset) {
    __syncthreads();
    for (int i = threadIdx.x; i < cw64; i += HTPB) {
      const uint64_t w = wcnt[i];
      if (w == wide_fill(UNOBS)) continue;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int c = 3 * i + k;
        const int64_t v = (int64_t)((w >> (WBITS * k)) & WMASK) - (int64_t)wide_bias(UNOBS);
        if (c < total && v) {
          atomicAdd(&counts[c], (unsigned long long)v);
          if (!UNOBS && !pres[c / a.length]) pres[c / a.length] = 1;
        }
      }
      if (reset) wcnt[i] = wide_fill(UNOBS);
    }
    __syncthreads();
  };
  // block iterations between drains: each counts at most HTPB * (VEC ? 2 * HU : 1) points, so no field
  // moves by more than the field's room (2^21 - 1 up from 0, 2^20 - 1 down from 2^20) in between
  const int64_t room = UNOBS ? (1 << 20) - 1 : (1 << 21) - 1;
  const int64_t stride = (int64_t)gridDim.x * HTPB;
  int since = 0;
  if (VEC) {
    const dv2* x2 = (const dv2*)x;
    const dv2* y2 = (const dv2*)y;
    const lv2* t2 = (const lv2*)t;
    const int64_t np = a.n >> 1;
    // software-pipelined: the next HU pairs per lane are in flight while the current ones are binned
    constexpr int HU = 2;
    // at least one block iteration between drains for the smaller (unobserve) room, or `since` never
    // meets drain_every and the packed fields carry into their neighbours
    static_assert(((1 << 20) - 1) / (HTPB * 2 * HU) - 1 >= 1, "WIDE drain schedule: HTPB * HU too large");
    const int drain_every = (int)(room / (HTPB * 2 * HU)) - 1;   // -1: the odd last row of block 0
    dv2 xa[HU], ya[HU];
    lv2 ta[HU];
    const int64_t p0 = (int64_t)blockIdx.x * HTPB;
    if (p0 < np) {   // uniform per block; below it every clamped index is a valid pair
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int64_t q = p0 + threadIdx.x + u * stride;
        const int64_t qc = q < np ? q : np - 1;   // unconditional loads (see below)
        xa[u] = ld_stream(&x2[qc]); ya[u] = ld_stream(&y2[qc]); ta[u] = ld_stream(&t2[qc]);
      }
    }
    // the loop bound is the block's first pair, so every thread of the block runs the same iterations
    // (the drains' barriers)
    for (int64_t pb = p0; pb < np; pb += HU * stride) {
      const int64_t p = pb + threadIdx.x, pn = p + HU * stride;
      dv2 xb[HU], yb[HU];
      lv2 tb[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        const int64_t q = pn + u * stride;
        // unconditional (clamped) loads: with the loads under a branch the compiler cannot count them and
        // waits for all outstanding loads (vmcnt(0)) before binning the current pairs, which serialises
        // this iteration's prefetch with its arithmetic
        const int64_t qc = q < np ? q : np - 1;
        xb[u] = ld_stream(&x2[qc]); yb[u] = ld_stream(&y2[qc]); tb[u] = ld_stream(&t2[qc]);
      }
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        if (p + u * stride < np) { one(xa[u].x, ya[u].x, ta[u].x); one(xa[u].y, ya[u].y, ta[u].y); }
        xa[u] = xb[u]; ya[u] = yb[u]; ta[u] = tb[u];
      }
      if (WIDE && ++since == drain_every) { drain(true); since = 0; }
    }
    if ((a.n & 1) && blockIdx.x == 0 && threadIdx.x == 0) one(x[a.n - 1], y[a.n - 1], t[a.n - 1]);
  } else {
    static_assert(((1 << 20) - 1) / HTPB >= 1, "WIDE drain schedule: HTPB too large");
    const int drain_every = (int)(room / HTPB);
    for (int64_t ib = (int64_t)blockIdx.x * HTPB; ib < a.n; ib += stride) {
      const int64_t i = ib + threadIdx.x;
      if (i < a.n) one(x[i], y[i], t[i]);
      if (WIDE && ++since == drain_every) { drain(true); since = 0; }
    }
  }
  if (skip) atomicAdd(&s_skip, skip);
  if (out) atomicAdd(&s_out, out);
  if (WIDE) {
    drain(false);
  } else {
    __syncthreads();
    for (int i = threadIdx.x; i < total; i += HTPB)
      if (cnt[i]) atomicAdd(&counts[i], (unsigned long long)(long long)cnt[i]);
    if (!UNOBS) {   // a row with a nonzero counter was seen by this workgroup
      for (int i = threadIdx.x; i < total; i += HTPB)
        if (cnt[i] && !pres[i / a.length]) pres[i / a.length] = 1;
      __syncthreads();
    }
  }
  if (!UNOBS) {
    for (int i = threadIdx.x; i < a.row_n; i += HTPB)
      if (pres[i] && !present[i]) present[i] = 1;
  }
  if (threadIdx.x == 0 && a.tally) {
    if (s_skip) atomicAdd(&tally[0], (unsigned long long)s_skip);
    if (s_out) atomicAdd(&tally[1], (unsigned long long)s_out);
  }
}

// histograms too large for LDS: 64-bit device atomics per feature
template <int PERIOD, bool UNOBS>
__global__ __launch_bounds__(256) void k_z3_hist_global(const double* __restrict__ x, const double* __restrict__ y,
                                                        const int64_t* __restrict__ t, HistArgs a,
                                                        uint8_t* __restrict__ present,
                                                        unsigned long long* __restrict__ counts,
                                                        unsigned long long* __restrict__ tally) {
  __shared__ int s_skip, s_out;
  if (threadIdx.x == 0) { s_skip = 0; s_out = 0; }
  __syncthreads();
  int skip = 0, out = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * 256) {
    int rb = 0;
    const int c = hist_slot<PERIOD, UNOBS>(x[i], y[i], t[i], a, rb, skip, out);
    if (c < 0) continue;
    if (UNOBS) {
      if (present[rb]) atomicAdd(&counts[c], ~0ull);  // += -1
    } else {
      atomicAdd(&counts[c], 1ull);
      if (!present[rb]) present[rb] = 1;
    }
  }
  if (skip) atomicAdd(&s_skip, skip);
  if (out) atomicAdd(&s_out, out);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_skip) atomicAdd(&tally[0], (unsigned long long)s_skip);
    if (s_out) atomicAdd(&tally[1], (unsigned long long)s_out);
  }
}

template <int PERIOD, bool UNOBS>
int launch_hist(gm_ctx* ctx, const double* x, const double* y, const int64_t* t, HistArgs a, uint8_t* present,
                unsigned long long* counts, unsigned long long* tally) {
  hipStream_t s = ctx->stream;
  // time-bin rows per LDS pass; every pass re-reads the 24 B/point, so more than HIST_MAX_PASSES
  // passes lose to the device-atomic kernel (measured: 2 LDS passes ~12 ms vs 45 ms atomics per 1B)
  // 32-bit LDS counters when every time-bin row fits one pass, else three 21-bit counters per 64-bit
  // word (WIDE): rows of `length` counters in (HIST_WIDE_BYTES / 8) words
  const int rows32 = (HIST_LDS_MAX) / (a.length + 1);
  const bool narrow = rows32 < a.n_bins;
  int rows = rows32;
  if (narrow) {
    auto bytes = [&](int64_t r) { return (r * a.length + 2) / 3 * 8 + r * 4; };
    rows = (int)std::min<int64_t>(a.n_bins, HIST_WIDE_BYTES / (a.length * 8 / 3 + 4) + 1);
    while (rows > 0 && bytes(rows) > HIST_WIDE_BYTES) --rows;
  }
  const int passes = rows > 0 ? (a.n_bins + rows - 1) / rows : 1 << 30;
  if (passes <= HIST_MAX_PASSES) {
    const bool vec = aligned16(x) && aligned16(y) && aligned16(t);
    int cus = 256;
    GM_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    for (int k = 0; k < passes; ++k) {
      a.row_lo = k * rows;
      a.row_n = std::min(rows, a.n_bins - a.row_lo);
      a.tally = k == 0;
      const int64_t tot = (int64_t)a.row_n * a.length;
      const int64_t cw64 = narrow ? (tot + 2) / 3 : (tot + 1) / 2;
      const size_t lds = (size_t)cw64 * 8 + (size_t)(a.row_n + 2048) * sizeof(int);
      const int per_cu = lds <= 72 * 1024 ? 2 : 1;  // 2 x 1024 threads is the CU's wave limit
      // per workgroup <= 2^31 increments so the int32 LDS counters cannot wrap
      const int64_t need = (a.n + (int64_t)2147483647 - 1) / (int64_t)2147483647;
      const int64_t want = (a.n + HTPB - 1) / HTPB;
      int64_t grid = std::min<int64_t>((int64_t)cus * per_cu, std::max<int64_t>(want, 1));
      grid = std::max(grid, need);
      if (ctx->hist_grid > 0) grid = std::max<int64_t>(ctx->hist_grid, need);   // GM_PARAM_HIST_GRID (drain tests)
      auto go = [&](auto kern) -> int {
        GM_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(HTPB), lds, s, x, y, t, a, present, counts, tally);
        GM_CHECK_LAUNCH();
        return GM_OK;
      };
      int rc;
      const bool top = a.top_s > 0;
      if (vec && top)
        rc = narrow ? go(k_z3_hist_lds<PERIOD, UNOBS, true, true, true>) : go(k_z3_hist_lds<PERIOD, UNOBS, true, false, true>);
      else if (vec)
        rc = narrow ? go(k_z3_hist_lds<PERIOD, UNOBS, true, true, false>) : go(k_z3_hist_lds<PERIOD, UNOBS, true, false, false>);
      else
        rc = narrow ? go(k_z3_hist_lds<PERIOD, UNOBS, false, true, false>) : go(k_z3_hist_lds<PERIOD, UNOBS, false, false, false>);
      if (rc) return rc;
    }
  } else {
    hipLaunchKernelGGL((k_z3_hist_global<PERIOD, UNOBS>), dim3((unsigned)std::min<int64_t>((a.n + 255) / 256, 256 * 16)),
                       dim3(256), 0, s, x, y, t, a, present, counts, tally);
    GM_CHECK_LAUNCH();
  }
  return GM_OK;
}

template <int PERIOD>
int launch_hist_p(gm_ctx* ctx, const double* x, const double* y, const int64_t* t, const HistArgs& a, bool unobs,
                  uint8_t* present, unsigned long long* counts, unsigned long long* tally) {
  return unobs ? launch_hist<PERIOD, true>(ctx, x, y, t, a, present, counts, tally)
               : launch_hist<PERIOD, false>(ctx, x, y, t, a, present, counts, tally);
}

}  // namespace gm

using namespace gm;

extern "C" {

int gm_z3_histogram(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n, int period,
                    int length, int unobserve, int bin_lo, int n_bins, uint8_t* present, int64_t* counts,
                    int64_t* tally) {
  if (!ctx || n < 0 || !valid_period(period) || length < 1 || n_bins < 1 || bin_lo < -32768 ||
      bin_lo + (int64_t)n_bins > 32768 || (int64_t)n_bins * length > ((int64_t)1 << 31) - 1)
    return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!x || !y || !t_ms || !present || !counts || !tally) return GM_E_INVALID;
  HistArgs a;
  a.n = n;
  a.length = length;
  a.bin_lo = bin_lo;
  a.n_bins = n_bins;
  a.row_lo = 0;
  a.row_n = n_bins;
  a.tally = 1;
  a.lon = lon_dim(21);
  a.lat = lat_dim(21);
  a.tim = time_dim(period, 21);
  // minZ / maxZ (Z3Histogram.scala:53-54): sfc.index(-180, -90, time.min) normalizes every dimension
  // to 0, sfc.index(180, 90, time.max) every dimension to maxIndex (x >= max, NormalizedDimension
  // .scala:60), so for every period minZ = 0 and maxZ = Z3(2^21-1, 2^21-1, 2^21-1) = Long.MaxValue
  a.zmin = 0;
  a.zmax = INT64_MAX;
  a.bsize = (double)(int64_t)((uint64_t)a.zmax - (uint64_t)a.zmin) / (double)length;
  {
    int e;
    a.inv_bsize = (std::frexp(a.bsize, &e) == 0.5 && e > -1000) ? std::ldexp(1.0, 1 - e) : 0.0;
  }
  a.top_s = a.top_sh = 0;
  if ((length & (length - 1)) == 0 && length <= (1 << 21)) {   // length 2^m: the TOP path
    int m = 0;
    while ((1 << m) < length) ++m;
    a.top_s = (63 - m) / 3;
    a.top_sh = 63 - m - 3 * a.top_s;
  }
  unsigned long long* c = (unsigned long long*)counts;
  unsigned long long* tl = (unsigned long long*)tally;
  const bool u = unobserve != 0;
  switch (period) {
    case DAY: return launch_hist_p<DAY>(ctx, x, y, t_ms, a, u, present, c, tl);
    case WEEK: return launch_hist_p<WEEK>(ctx, x, y, t_ms, a, u, present, c, tl);
    case MONTH: return launch_hist_p<MONTH>(ctx, x, y, t_ms, a, u, present, c, tl);
    default: return launch_hist_p<YEAR>(ctx, x, y, t_ms, a, u, present, c, tl);
  }
}

}  // extern "C"
