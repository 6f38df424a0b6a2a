// gm_ranges.hip -- batched range decomposition: ZN.zranges (Z2/Z3) and XZ2/XZ3 ranges on gfx950.
//
// Z curves: one 256-thread workgroup per query (k_zranges).  XZ curves: one 64-lane wave per query
// (k_xzranges_w, below).  The Scala code walks a FIFO queue one node at a time (ZN.scala:193-218,
// XZ2SFC.scala:205-227) and its maxRanges budget truncates at an exact FIFO position.  Here a whole
// tree level is processed in parallel and the FIFO semantics are reconstructed with prefix sums:
//
//   Z curves   after node i of a level the queue holds (K-i-1) level nodes + the queued children,
//              so the budget fires at the first i with
//                 nR + CC(i) + CO(i) + (K - i - 1) >= rangeStop          (ZN.scala:214)
//              (CC/CO = inclusive counts of contained / overlapping children).  Nodes after i are
//              bottomed out as overlapping ranges at their own level, queued children at theirs.
//   XZ curves  the budget is checked before every element (ranges.size < rangeStop,
//              XZ2SFC.scala:205), so the first unprocessed element is the first i with
//                 nR + A(i-1) >= rangeStop        (A = inclusive count of non-disjoint elements);
//              bottom-out emits full intervals at the current and the next level (:219-227).
//
// Z: emitted ranges are tree nodes that never nest, so after the walk they are disjoint; a merge of
// the walk's sorted runs by rank (or an LDS bitonic sort) followed by a parallel adjacency merge
// reproduces the sort + merge of ZN.scala:221-241 exactly.  XZ: the sorted order follows from subtree
// counts (no comparison sort) and the merge is a ballot per 64 ranges (XZ2SFC.scala:231-249).
//
// Frontier and range lists live in per-query global workspaces (HBM is plentiful); the zbounds /
// normalized query windows sit in LDS.
#include <string.h>

#include <algorithm>
#include <vector>

#include "gm_internal.hpp"
#include "gm_scan.hpp"

namespace gm {

#ifndef GM_RTPB
#define GM_RTPB 512
#endif
constexpr int RTPB = GM_RTPB;   // threads per query (one workgroup each)
constexpr int RNW = RTPB / 64;
constexpr int MAXB = 256;       // zbounds / windows per query
#ifndef GM_LDS_SORT
#define GM_LDS_SORT 4096
#endif
constexpr int LDS_SORT = GM_LDS_SORT;  // ranges sorted in LDS; larger lists sort in global memory
#define GM_XZ_BOUNDS __launch_bounds__(RTPB)

enum : int32_t { QS_OK = 0, QS_OUT_OF_BOUNDS = 1, QS_UNORDERED = 3, QS_CAPACITY = 4, QS_TOO_MANY_BOUNDS = 5 };

// ------------------------------------------------------------------ block helpers

__device__ __forceinline__ int64_t block_exscan(int64_t v, int64_t* s_tmp, int64_t& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_tmp[w] = x;
  __syncthreads();
  int64_t pre = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < RNW; ++k) {
    const int64_t t = s_tmp[k];
    if (k < w) pre += t;
    tot += t;
  }
  __syncthreads();
  total = tot;
  return pre + x - v;
}

// Java `(1L << s) - 1` with the shift distance masked to 6 bits
__device__ __forceinline__ int64_t low_mask(int s) { return (int64_t)(((uint64_t)1 << (s & 63)) - 1u); }
__device__ __forceinline__ int64_t jshl(int64_t v, int s) { return (int64_t)((uint64_t)v << (s & 63)); }

template <int D>
__device__ __forceinline__ int32_t zdim(int64_t z, int d) {
  return D == 3 ? z3_combine(z >> d) : z2_combine(z >> d);
}

// Z3.contains / Z2.contains (Z3.scala:93-98, Z2.scala:80-83) on decoded dims
template <int D>
__device__ __forceinline__ bool z_contains(const int32_t* b, int64_t v) {
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int32_t x = zdim<D>(v, d);
    if (!(x >= b[d] && x <= b[D + d])) return false;
  }
  return true;
}

// bitonic sort of (key, idx) pairs, P a power of two, keys padded with INT64_MAX
template <class K, class I>
__device__ void bitonic(K* key, I* idx, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += RTPB) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const int64_t a = key[i], b = key[ixj];
          if ((a > b) == up) {
            key[i] = b; key[ixj] = a;
            const auto t = idx[i]; idx[i] = idx[ixj]; idx[ixj] = t;
          }
        }
      }
      __syncthreads();
    }
  }
}

constexpr int MAXRUNS = 64;   // sorted runs merged by rank; more fall back to the bitonic sort

// rank of `key` among run [lo, hi) of keys: elements < key (or <= key when `le`)
__device__ __forceinline__ int run_rank(const int64_t* keys, int lo, int hi, int64_t key, bool le) {
  int a = lo, b = hi;
  while (a < b) {
    const int m = (a + b) >> 1;
    const int64_t v = keys[m];
    if (v < key || (le && v == key)) a = m + 1;
    else b = m;
  }
  return a - lo;
}

// Sort the n ranges of this query by lower and merge adjacent ones into out (ZN.scala:221-241);
// returns the merged count (same on every thread).  The walk emits each tree level in curve order
// (children are generated in quadrant order from a curve-ordered frontier, and bottom-out appends
// ordered frontiers), so the list is a concatenation of a few ascending runs: they are merged by
// rank -- each range's sorted position is its offset in its run plus its rank in every other run,
// found by binary search (stable: ties rank after earlier runs) -- with one barrier.  A list with
// more than MAXRUNS runs takes the bitonic sort.
__device__ int sort_merge(const int64_t* rlo, const int64_t* rhi, const uint8_t* rc, int n, int64_t* gkey,
                          int32_t* gidx, gm_range* out, int64_t* s_key, int16_t* s_idx, int64_t* s_tmp) {
  __shared__ int s_run[MAXRUNS + 1];
  if (n == 0) return 0;
  const bool lds = n <= LDS_SORT;
  // run starts: rlo[j] < rlo[j - 1]
  if (threadIdx.x == 0) s_run[0] = 0;
  __syncthreads();
  int64_t nrun = 1;
  for (int c = 0; c < n && nrun <= MAXRUNS; c += RTPB) {
    const int j = c + threadIdx.x;
    const int f = (j > 0 && j < n && rlo[j] < rlo[j - 1]) ? 1 : 0;
    int64_t tot;
    const int64_t ex = block_exscan(f, s_tmp, tot);
    if (f && nrun + ex < MAXRUNS) s_run[nrun + ex] = j;
    nrun += tot;
    if (lds && j < n) s_key[j] = rlo[j];
  }
  __syncthreads();
  if (nrun <= MAXRUNS) {
    const int R = (int)nrun;
    if (threadIdx.x == 0) s_run[R] = n;
    __syncthreads();
    const int64_t* keys = lds ? s_key : rlo;
    for (int j = threadIdx.x; j < n; j += RTPB) {
      int r = 0;
      while (r + 1 < R && s_run[r + 1] <= j) ++r;   // R is small: linear scan
      const int64_t key = keys[j];
      int pos = j - s_run[r];
      for (int r2 = 0; r2 < R; ++r2)
        if (r2 != r) pos += run_rank(keys, s_run[r2], s_run[r2 + 1], key, r2 < r);
      if (lds) s_idx[pos] = (int16_t)j;
      else gidx[pos] = j;
    }
    __syncthreads();
  } else {
    int P = 1;
    while (P < n) P <<= 1;
    const bool lp = P <= LDS_SORT;
    for (int i = threadIdx.x; i < P; i += RTPB) {
      const int64_t k = i < n ? rlo[i] : INT64_MAX;
      if (lp) { s_key[i] = k; s_idx[i] = (int16_t)i; }
      else { gkey[i] = k; gidx[i] = i; }
    }
    __syncthreads();
    if (lp) bitonic(s_key, s_idx, P);
    else bitonic(gkey, gidx, P);
  }
  // run starts: lower > previous upper + 1 (Java long wrap); sorted disjoint ranges have increasing
  // uppers, so the previous upper is the merged run's max (ZN.scala:228-230)
  int64_t* run_of = lds ? s_key : gkey;  // keys are dead after the sort: reuse for run ids
  int64_t base = 0;
  for (int c = 0; c < n; c += RTPB) {
    const int j = c + threadIdx.x;
    int start = 0, src = 0;
    if (j < n) {
      src = lds ? (int)(uint16_t)s_idx[j] : gidx[j];
      if (j == 0) start = 1;
      else {
        const int prev = lds ? (int)(uint16_t)s_idx[j - 1] : gidx[j - 1];
        start = !(rlo[src] <= (int64_t)((uint64_t)rhi[prev] + 1u));
      }
    }
    int64_t tot;
    const int64_t ex = block_exscan(start, s_tmp, tot);
    if (j < n) {
      const int64_t run = base + ex + start - 1;
      run_of[j] = run;
      if (start) { out[run].lower = rlo[src]; out[run].contained = 1; out[run].reserved = 0; }
      bool last = (j == n - 1);
      if (!last) {
        const int nx = lds ? (int)(uint16_t)s_idx[j + 1] : gidx[j + 1];
        last = !(rlo[nx] <= (int64_t)((uint64_t)rhi[src] + 1u));
      }
      if (last) out[run].upper = rhi[src];
    }
    base += tot;
  }
  __syncthreads();
  // contained = AND over the run
  for (int j = threadIdx.x; j < n; j += RTPB) {
    const int src = lds ? (int)(uint16_t)s_idx[j] : gidx[j];
    if (!rc[src]) out[run_of[j]].contained = 0;
  }
  __syncthreads();
  const int total_runs = (int)base;
  return total_runs;
}

// Batch output: every query's merged ranges are appended to one device buffer (one atomic per query)
// with their (start, count) recorded by query index; the host driver then scans the counts and
// gathers the buffer into query order.  Phase 2 re-runs the queries whose first-pass workspace
// overflowed, through qmap.
struct BatchOut {
  const int32_t* qmap;           // block -> query index (phase 2), null: q0 + block
  int64_t ocap;                  // stride of the per-block merged scratch (a.out), ranges
  gm_range* dbuf;                // batch buffer
  int64_t dcap;
  unsigned long long* total;
  int64_t* start;                // per query
  int32_t* count;
  int32_t* status;
};

__device__ __forceinline__ int64_t batch_query(const BatchOut& bo, int64_t q0, int64_t qc) {
  return bo.qmap ? (int64_t)bo.qmap[qc] : q0 + qc;
}

// record a query's result (every thread of the block calls it; `ws` = its m merged ranges)
__device__ void batch_finish(const BatchOut& bo, int64_t q, int m, int status, const gm_range* ws) {
  __shared__ unsigned long long s_base;
  if (threadIdx.x == 0) {
    s_base = (status == QS_OK && m > 0) ? atomicAdd(bo.total, (unsigned long long)m) : 0ull;
    bo.start[q] = (int64_t)s_base;
    bo.count[q] = status == QS_OK ? m : 0;
    bo.status[q] = status;
  }
  __syncthreads();
  if (status == QS_OK)
    for (int j = threadIdx.x; j < m; j += RTPB)
      if ((int64_t)s_base + j < bo.dcap) bo.dbuf[s_base + j] = ws[j];
}

// ------------------------------------------------------------------ Z ranges kernel

struct ZRangesArgs {
  const int32_t* box_off;   // [nq + 1]
  const double* xy;         // 4 per box
  const int32_t* time_off;  // [nq + 1] (Z3 only)
  const int64_t* t;         // 2 per interval
  const int32_t* zb_off;    // raw ZRange mode (gm_zranges): [nq + 1] bound offsets, else null
  const int64_t* zb;        //   (min, max) per bound
  int64_t q0;               // first query of this chunk
  NDim lon, lat, tim;
  int range_precision, range_stop, recurse_stop;
  int64_t fcap, rcap;
  int64_t* fa;              // frontier ping / pong, 2 x fcap per query
  int64_t* rlo;
  int64_t* rhi;
  uint8_t* rc;
  int64_t* gkey;
  int32_t* gidx;
  gm_range* out;            // merged ranges scratch, bo.ocap per block
  BatchOut bo;
};

template <int D>
__global__ __launch_bounds__(RTPB) void k_zranges(ZRangesArgs a) {
  __shared__ int64_t s_zb[2 * MAXB];
  __shared__ int32_t s_dim[2 * D * MAXB];  // decoded min dims, max dims per bound
  __shared__ int64_t s_tmp[RNW];
  __shared__ int s_err, s_stop;
  __shared__ int64_t s_prefix;
  __shared__ int s_common;
  __shared__ int64_t s_key[LDS_SORT];
  __shared__ int16_t s_idx[LDS_SORT];

  const int64_t qc = blockIdx.x;            // query within the chunk
  const int64_t q = batch_query(a.bo, a.q0, qc);
  int64_t* F = a.fa + qc * 2 * a.fcap;      // F, G adjacent per query (the merged output aliases them)
  int64_t* G = F + a.fcap;
  int64_t* rlo = a.rlo + qc * a.rcap;
  int64_t* rhi = a.rhi + qc * a.rcap;
  uint8_t* rc = a.rc + qc * a.rcap;

  const bool raw = a.zb != nullptr;
  const int b0 = raw ? a.zb_off[q] : a.box_off[q];
  const int nbx = (raw ? a.zb_off[q + 1] : a.box_off[q + 1]) - b0;
  int t0 = 0, ntm = 1;
  if (D == 3 && !raw) { t0 = a.time_off[q]; ntm = a.time_off[q + 1] - t0; }
  const int nb = nbx * ntm;
  if (threadIdx.x == 0) s_err = (nb > MAXB) ? QS_TOO_MANY_BOUNDS : QS_OK;
  __syncthreads();
  if (s_err || nb <= 0) {
    batch_finish(a.bo, q, 0, s_err, nullptr);
    return;
  }
  // zbounds: Z3SFC.ranges builds ZRange(index(xmin, ymin, tmin), index(xmax, ymax, tmax)) for the
  // cross product xy x t, non-lenient (Z3SFC.scala:63-65); Z2SFC.ranges likewise (Z2SFC.scala:50)
  for (int j = threadIdx.x; j < nb; j += RTPB) {
    int64_t lo = 0, hi = 0;
    uint8_t st = ST_OK;
    if (raw) {   // ZN.zranges(Array[ZRange], ...) (ZN.scala:110-113): the bounds as given
      lo = a.zb[2 * (int64_t)(b0 + j)];
      hi = a.zb[2 * (int64_t)(b0 + j) + 1];
    } else if (D == 3) {
      const double* bx = a.xy + 4 * (int64_t)(b0 + j / ntm);
      const int64_t* tt = a.t + 2 * (int64_t)(t0 + j % ntm);
      auto idx = [&](double x, double y, int64_t tv, int64_t& z) -> uint8_t {
        const double td = (double)tv;
        if (!(x >= a.lon.min && x <= a.lon.max && y >= a.lat.min && y <= a.lat.max && td >= a.tim.min &&
              td <= a.tim.max))
          return ST_OUT_OF_BOUNDS;
        z = z3_apply(normalize(a.lon, x), normalize(a.lat, y), normalize(a.tim, td));
        return ST_OK;
      };
      st = idx(bx[0], bx[1], tt[0], lo);
      if (!st) st = idx(bx[2], bx[3], tt[1], hi);
    } else {
      const double* bx = a.xy + 4 * (int64_t)(b0 + j);
      auto idx = [&](double x, double y, int64_t& z) -> uint8_t {
        if (!(x >= a.lon.min && x <= a.lon.max && y >= a.lat.min && y <= a.lat.max)) return ST_OUT_OF_BOUNDS;
        z = z2_apply(normalize(a.lon, x), normalize(a.lat, y));
        return ST_OK;
      };
      st = idx(bx[0], bx[1], lo);
      if (!st) st = idx(bx[2], bx[3], hi);
    }
    if (!st && lo > hi) st = QS_UNORDERED;  // ZRange require(min <= max) (package.scala:24)
    if (st) atomicMax(&s_err, (int)st);
    s_zb[2 * j] = lo;
    s_zb[2 * j + 1] = hi;
    for (int d = 0; d < D; ++d) {
      s_dim[(2 * D) * j + d] = zdim<D>(lo, d);
      s_dim[(2 * D) * j + D + d] = zdim<D>(hi, d);
    }
  }
  __syncthreads();
  if (s_err) {
    batch_finish(a.bo, q, 0, s_err, nullptr);
    return;
  }
  // longestCommonPrefix (ZN.scala:272-281)
  if (threadIdx.x == 0) {
    const int total_bits = D == 3 ? 63 : 62;
    int shift = total_bits - D;
    int64_t head = (int64_t)((uint64_t)s_zb[0] >> (shift & 63));
    for (;;) {
      bool all = true;
      for (int i = 1; i < 2 * nb; ++i)
        if ((int64_t)((uint64_t)s_zb[i] >> (shift & 63)) != head) { all = false; break; }
      if (!(all && shift > -1)) break;
      shift -= D;
      head = (int64_t)((uint64_t)s_zb[0] >> (shift & 63));
    }
    shift += D;
    s_prefix = s_zb[0] & jshl(INT64_MAX, shift);
    s_common = 64 - shift;
  }
  __syncthreads();

  auto is_contained = [&](int64_t mn, int64_t mx) {
    for (int i = 0; i < nb; ++i)
      if (z_contains<D>(&s_dim[2 * D * i], mn) && z_contains<D>(&s_dim[2 * D * i], mx)) return true;
    return false;
  };
  auto is_overlapped = [&](int64_t mn, int64_t mx) {
    for (int i = 0; i < nb; ++i) {
      const int32_t* b = &s_dim[2 * D * i];
      bool ok = true;
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int32_t v1 = zdim<D>(mn, d), v2 = zdim<D>(mx, d);
        const int32_t lo = b[d] > v1 ? b[d] : v1, hi = b[D + d] < v2 ? b[D + d] : v2;
        ok = ok && (lo <= hi);
      }
      if (ok) return true;
    }
    return false;
  };

  const int64_t range_stop = a.range_stop;
  int offset = 64 - s_common;
  int64_t nR = 0, K = 0;
  // initial level: checkValue(commonPrefix, 0) (ZN.scala:183)
  if (threadIdx.x == 0) {
    const int64_t mn = s_prefix, mx = mn | low_mask(offset);
    if (is_contained(mn, mx) || offset < 64 - a.range_precision) {
      rlo[0] = mn; rhi[0] = mx; rc[0] = 1; s_stop = 1;
    } else if (is_overlapped(mn, mx)) {
      F[0] = mn; s_stop = 2;
    } else {
      s_stop = 0;
    }
  }
  __syncthreads();
  if (s_stop == 1) nR = 1;
  if (s_stop == 2) K = 1;
  offset -= D;
  int level = 0;
  bool done = (K == 0);
  int err = QS_OK;
  while (!done) {
    // process level: K nodes in F at child offset `offset`; children -> G
    int64_t cc_carry = 0, co_carry = 0;
    int64_t stop_at = -1;
    for (int64_t c = 0; c < K; c += RTPB) {
      const int64_t i = c + threadIdx.x;
      uint32_t cmask = 0, omask = 0;
      int64_t p = 0;
      if (i < K) {
        p = F[i];
        for (int qd = 0; qd < (1 << D); ++qd) {
          const int64_t mn = p | jshl(qd, offset);
          const int64_t mx = mn | low_mask(offset);
          if (is_contained(mn, mx) || offset < 64 - a.range_precision) cmask |= 1u << qd;
          else if (is_overlapped(mn, mx)) omask |= 1u << qd;
        }
      }
      const int cc = __popc(cmask), co = __popc(omask);
      int64_t pt;   // one scan of (contained | overlapping << 32)
      const int64_t px = block_exscan((int64_t)cc | ((int64_t)co << 32), s_tmp, pt);
      const int64_t ccx = px & 0xffffffff, cox = px >> 32, cct = pt & 0xffffffff, cot = pt >> 32;
      // budget (ZN.scala:214) after node i; bounded above by the chunk totals at its first node
      int sl = INT32_MAX;
      if (nR + cc_carry + cct + co_carry + cot + (K - c - 1) >= range_stop) {
        if (threadIdx.x == 0) s_stop = INT32_MAX;
        __syncthreads();
        if (i < K) {
          const int64_t f = nR + cc_carry + ccx + cc + co_carry + cox + co + (K - i - 1);
          if (f >= range_stop) atomicMin(&s_stop, (int)threadIdx.x);
        }
        __syncthreads();
        sl = s_stop;
      }
      const bool emit = (i < K) && (sl == INT32_MAX || (int)threadIdx.x <= sl);
      if (emit) {
        int64_t rpos = nR + cc_carry + ccx, fpos = co_carry + cox;
        if (rpos + cc > a.rcap || fpos + co > a.fcap) {
          atomicMax(&s_err, QS_CAPACITY);
        } else {
          for (int qd = 0; qd < (1 << D); ++qd) {
            const int64_t mn = p | jshl(qd, offset);
            if (cmask >> qd & 1) { rlo[rpos] = mn; rhi[rpos] = mn | low_mask(offset); rc[rpos] = 1; ++rpos; }
            else if (omask >> qd & 1) { G[fpos++] = mn; }
          }
        }
      }
      if (sl != INT32_MAX) {
        // counts up to and including node c + sl
        __shared__ int64_t s_cc_upto, s_co_upto;
        if ((int)threadIdx.x == sl) { s_cc_upto = cc_carry + ccx + cc; s_co_upto = co_carry + cox + co; }
        __syncthreads();
        stop_at = c + sl;
        cc_carry = s_cc_upto;
        co_carry = s_co_upto;
        break;
      }
      cc_carry += cct;
      co_carry += cot;
      __syncthreads();
    }
    __syncthreads();
    if (s_err) { err = s_err; break; }
    if (stop_at >= 0) {
      // bottomOut (ZN.scala:173-180): rest of this level, then the queued children, as overlapping
      int64_t pos = nR + cc_carry;
      const int64_t rest = K - stop_at - 1, kids = co_carry;
      if (pos + rest + kids > a.rcap) { err = QS_CAPACITY; break; }
      for (int64_t j = threadIdx.x; j < rest; j += RTPB) {
        const int64_t mn = F[stop_at + 1 + j];
        rlo[pos + j] = mn; rhi[pos + j] = mn | low_mask(offset + D); rc[pos + j] = 0;
      }
      pos += rest;
      for (int64_t j = threadIdx.x; j < kids; j += RTPB) {
        const int64_t mn = G[j];
        rlo[pos + j] = mn; rhi[pos + j] = mn | low_mask(offset); rc[pos + j] = 0;
      }
      nR = pos + kids;
      break;
    }
    nR += cc_carry;
    K = co_carry;
    if (K == 0) break;
    // level terminator (ZN.scala:195-205)
    level += 1;
    offset -= D;
    int64_t* tmp = F; F = G; G = tmp;
    if (level >= a.recurse_stop || offset < 0) {
      if (nR + K > a.rcap) { err = QS_CAPACITY; break; }
      for (int64_t j = threadIdx.x; j < K; j += RTPB) {
        const int64_t mn = F[j];
        rlo[nR + j] = mn; rhi[nR + j] = mn | low_mask(offset + D); rc[nR + j] = 0;
      }
      nR += K;
      break;
    }
    __syncthreads();
  }
  __syncthreads();
  if (err) {
    batch_finish(a.bo, q, 0, err, nullptr);
    return;
  }
  gm_range* ws = a.out + qc * a.bo.ocap;
  const int m = sort_merge(rlo, rhi, rc, (int)nR, a.gkey + qc * a.rcap, a.gidx + qc * a.rcap, ws, s_key, s_idx, s_tmp);
  batch_finish(a.bo, q, m, QS_OK, ws);
}

}  // namespace gm

namespace gm {

// ------------------------------------------------------------------ XZ ranges kernel

// element (ix, iy[, iz]) at level L packed 30 (XZ2) / 20 (XZ3) bits per coordinate
template <int D>
__device__ __forceinline__ uint32_t xcoord(uint64_t e, int d) {
  return D == 2 ? (uint32_t)((e >> (30 * d)) & 0x3fffffffu) : (uint32_t)((e >> (20 * d)) & 0xfffffu);
}
template <int D>
__device__ __forceinline__ uint64_t xpack(const uint32_t* c) {
  uint64_t e = 0;
  for (int d = 0; d < D; ++d) e |= (uint64_t)c[d] << ((D == 2 ? 30 : 20) * d);
  return e;
}

// child k of an element, XElement.children order: bit d of k takes the upper half of dimension d
// (XZ2SFC.scala:406-415, XZ3SFC.scala:449-464)
template <int D>
__device__ __forceinline__ uint64_t xchild(uint64_t p, int k) {
  uint32_t c[3];
  for (int d = 0; d < D; ++d) c[d] = 2 * xcoord<D>(p, d) + ((k >> d) & 1);
  return xpack<D>(c);
}

// sequenceCode (XZ2SFC.scala:264-286, XZ3SFC.scala:275-304) of an element's lower corner: the
// descent compares x < xCenter at every level, i.e. reads the element's coordinate bits MSB first
template <int D>
__device__ __forceinline__ int64_t xseq(uint64_t e, int L, int g) {
  const int sh = D == 2 ? 2 : 3;
  int64_t step = (((int64_t)1 << (sh * g)) - 1) / ((1 << D) - 1);
  int64_t cs = 0;
  for (int i = 0; i < L; ++i) {
    const int b = L - 1 - i;
    int qd = 0;
    for (int d = 0; d < D; ++d) qd |= (int)((xcoord<D>(e, d) >> b) & 1u) << d;
    cs += 1 + (int64_t)qd * step;
    step = (step - 1) >> sh;
  }
  return cs;
}
// sequenceInterval full width: (base^(g - L + 1) - 1) / (base - 1) (XZ2SFC.scala:303)
template <int D>
__device__ __forceinline__ int64_t xspan(int L, int g) {
  const int sh = D == 2 ? 2 : 3;
  return (((int64_t)1 << (sh * (g - L + 1))) - 1) / ((1 << D) - 1);
}

// ------------------------------------------------------------------ XZ ranges: one wave per query
// XZ2SFC.ranges / XZ3SFC.ranges (XZ2SFC.scala:130-252, XZ3SFC.scala:139-262) for a batch of queries,
// one 64-lane wave each, with no block barrier anywhere (a 512-thread workgroup per query was bound by
// its barriers: most queries emit only 38-388 ranges).
//
//  1. walk: the FIFO queue of the reference is processed level by level.  Level L's elements are the
//     2^D children (XElement.children order) of the overlapping elements of level L - 1 (its
//     "parents", in queue order; level 1 = the children of the unit element).  Each is classified
//     disjoint (0) / contained (1) / overlapping (2, its children queued) in chunks of 64 lanes, and the
//     budget -- element i is processed only while ranges.size < rangeStop (XZ2SFC.scala:205), i.e.
//     nR + (non-disjoint elements before i) < rangeStop -- is a ballot + mbcnt prefix.  From the first
//     unprocessed element on, every element of the level is bottomed out as its full interval (3,
//     :219-227), and so are the queued children of the level's overlapping elements: each of those
//     parents' children chain (a child's full-interval upper is its next sibling's lower) into exactly
//     the parent's own full interval, merged with its point interval [cs, cs] -- so such a parent is
//     recorded as kind 3 itself.  Reaching level g (`while (level < g ...)`) bottoms out the same way.
//  2. order: the emitted ranges are tree nodes whose sequence codes are in DFS preorder (a parent's
//     point interval, then its children's subtrees in child order), so the sorted position of every
//     range follows from subtree counts: an up-sweep over the levels gives each parent T = 1 (its own
//     point interval; 0 for the unit element) + the ranges of its children's subtrees, a down-sweep
//     gives each element its position.  No comparison sort.
//  3. merge: adjacent ranges merge when lower <= previous upper + 1 (Java long wrap), contained = AND
//     (XZ2SFC.scala:231-249), with ballots over 64 sorted ranges at a time, written straight into the
//     batch buffer.
// Per query (global workspace, XzWs): parents of all levels (packed coordinates), T / B per parent,
// per element kind << 30 | the global parent id of an overlapping element, the pre-merge ranges, and
// the normalized windows.
constexpr int XW_TPB = 256;   // 4 waves (= 4 queries) per workgroup
constexpr int XW_MAXL = 32;   // levels (g <= 29)

struct XzWs {   // byte offsets of one query's arrays within its stride
  int64_t pcap, ecap, rcap;
  int64_t o_par, o_tb, o_pi, o_ek, o_lo, o_hi, o_rc, o_win, stride;
};

__host__ __device__ inline XzWs xz_ws(int D, int64_t pcap, int64_t rcap) {
  XzWs w{};
  auto al = [](int64_t v) { return (v + 15) & ~(int64_t)15; };
  w.pcap = pcap; w.ecap = pcap << D; w.rcap = rcap;
  w.o_par = 0;
  w.o_tb = w.o_par + al(pcap * 8);
  w.o_pi = w.o_tb + al(pcap * 4);
  w.o_ek = w.o_pi + al(pcap * 4);
  w.o_lo = w.o_ek + al(w.ecap * 4);
  w.o_hi = w.o_lo + al(rcap * 8);
  w.o_rc = w.o_hi + al(rcap * 8);
  w.o_win = w.o_rc + al(rcap);
  w.stride = w.o_win + al((int64_t)2 * D * MAXB * 8);
  return w;
}

struct XZWaveArgs {
  const int32_t* win_off;   // [nq + 1]
  const double* win;        // 2*D doubles per window, user space (mins then maxs)
  int64_t q0, m;            // first query of this launch, queries in it
  int g;
  double zhi;               // XZ3 z upper bound (maxOffset(period))
  int range_stop;
  XzWs ws;
  char* base;               // m query strides
  BatchOut bo;
};

__device__ __forceinline__ void wave_mem_sync() {   // this wave's global stores visible to its own lanes
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// waves per SIMD: 6 for XZ2 (80 VGPRs, a few spills off the hot path) and 5 for XZ3 (96): 3.26-3.34 ->
// 3.04-3.10 and 10.50-10.63 -> 9.88-9.97 ms per 100k queries into HBM against the compiler's choice
// (89 / 103 VGPRs, 5 / 4 waves); 6 for XZ3 spilled more and ran 10.6-10.8 (profiles/r6/xz_ranges_occupancy_ab.txt)
template <int D>
__global__ __launch_bounds__(XW_TPB) __attribute__((amdgpu_waves_per_eu(D == 2 ? 6 : 5))) void k_xzranges_w(XZWaveArgs a) {
  constexpr int NK = 1 << D;
  __shared__ int32_t s_lb[XW_TPB / 64][XW_MAXL + 1], s_le[XW_TPB / 64][XW_MAXL + 1], s_lnp[XW_TPB / 64][XW_MAXL + 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t qc = (int64_t)blockIdx.x * (XW_TPB / 64) + wv;
  if (qc >= a.m) return;   // whole wave
  const int64_t q = batch_query(a.bo, a.q0, qc);
  const XzWs W = a.ws;
  char* qb = a.base + qc * W.stride;
  uint64_t* par = (uint64_t*)(qb + W.o_par);
  uint32_t* tb = (uint32_t*)(qb + W.o_tb);
  uint32_t* pix = (uint32_t*)(qb + W.o_pi);
  uint32_t* ek = (uint32_t*)(qb + W.o_ek);
  int64_t* rlo = (int64_t*)(qb + W.o_lo);
  int64_t* rhi = (int64_t*)(qb + W.o_hi);
  uint8_t* rcb = (uint8_t*)(qb + W.o_rc);
  double* wn = (double*)(qb + W.o_win);
  int32_t* lb = s_lb[wv];
  int32_t* le = s_le[wv];
  int32_t* lnp = s_lnp[wv];
  const int g = a.g;
  auto finish = [&](int64_t base, int64_t m, int st) {
    if (lane == 0) {
      a.bo.start[q] = base;
      a.bo.count[q] = st == QS_OK ? (int32_t)m : 0;
      a.bo.status[q] = st;
    }
  };

  // windows, normalized non-lenient (XZ2SFC.scala:132-135 / XZ3SFC.scala:142-145 -> normalize)
  const int w0 = a.win_off[q], nw = a.win_off[q + 1] - w0;
  if (nw > MAXB) { finish(0, 0, QS_TOO_MANY_BOUNDS); return; }
  if (nw <= 0) { finish(0, 0, QS_OK); return; }
  int werr = QS_OK;
  for (int j = lane; j < nw; j += 64) {
    const double* w = a.win + 2 * D * (int64_t)(w0 + j);
    const double lo[3] = {-180.0, -90.0, 0.0}, hi[3] = {180.0, 90.0, a.zhi};
    bool ordered = true, inb = true;
    for (int d = 0; d < D; ++d) {
      ordered = ordered && (w[d] <= w[D + d]);
      inb = inb && (w[d] >= lo[d]) && (w[D + d] <= hi[d]);
    }
    if (!ordered) werr = max(werr, (int)QS_UNORDERED);
    else if (!inb) werr = max(werr, (int)QS_OUT_OF_BOUNDS);
    for (int d = 0; d < D; ++d) {
      const double size = __dsub_rn(hi[d], lo[d]);
      wn[2 * D * j + d] = __ddiv_rn(__dsub_rn(w[d], lo[d]), size);
      wn[2 * D * j + D + d] = __ddiv_rn(__dsub_rn(w[D + d], lo[d]), size);
    }
  }
  for (int o = 32; o > 0; o >>= 1) werr = max(werr, __shfl_xor(werr, o, 64));
  if (werr) { finish(0, 0, werr); return; }
  wave_mem_sync();
  // one window (the common case) stays in registers
  double W1[2 * D];
  if (nw == 1)
    for (int k = 0; k < 2 * D; ++k) W1[k] = wn[k];
  auto classify = [&](uint64_t e, double len) -> int {   // 0 disjoint, 1 contained, 2 overlapping
    double mn[D], ext[D];
    for (int d = 0; d < D; ++d) {
      const double ci = (double)xcoord<D>(e, d);
      mn[d] = __dmul_rn(ci, len);                    // xmin
      ext[d] = __dmul_rn(__dadd_rn(ci, 2.0), len);   // xext = xmax + length
    }
    if (nw == 1) {
      bool c = true, o = true;
      for (int d = 0; d < D; ++d) {
        c = c && (W1[d] <= mn[d]) && (W1[D + d] >= ext[d]);   // XElement.isContained (XZ2SFC.scala:400-401)
        o = o && (W1[D + d] >= mn[d]) && (W1[d] <= ext[d]);   // XElement.overlaps (XZ2SFC.scala:403-404)
      }
      return c ? 1 : (o ? 2 : 0);
    }
    bool ovl = false;
    for (int w = 0; w < nw; ++w) {
      const double* Wp = wn + 2 * D * w;
      bool c = true, o = true;
      for (int d = 0; d < D; ++d) {
        const double lo = Wp[d], hi = Wp[D + d];
        c = c && (lo <= mn[d]) && (hi >= ext[d]);
        o = o && (hi >= mn[d]) && (lo <= ext[d]);
      }
      if (c) return 1;
      ovl = ovl || o;
    }
    return ovl ? 2 : 0;
  };

  // ---- 1. walk
  if (lane == 0) { par[0] = 0; lb[1] = 0; le[1] = 0; lnp[1] = 1; }
  wave_mem_sync();
  int64_t nP = 1, eb = 0, nR = 0;
  int L = 1, Lmax = 1, err = QS_OK;
  const int64_t rs = a.range_stop;
  for (;; ++L) {
    const int64_t np = lnp[L], K = np << D, pb = lb[L];
    const bool last = L >= g;   // never processed (level < g fails): bottomed out as full intervals
    const double len = ldexp(1.0, -L);
    int64_t cA = 0, c2 = 0, stop_at = last ? 0 : -1;
    for (int64_t c = 0; c < K; c += 64) {
      const int64_t i = c + lane;
      const bool act = i < K;
      int kind = 0;
      if (act && stop_at < 0) kind = classify(xchild<D>(par[pb + (i >> D)], (int)(i & (NK - 1))), len);
      if (stop_at < 0) {
        const uint64_t nd = __ballot(act && kind != 0);
        const int64_t excl = cA + lanes_below(nd);
        const uint64_t over = __ballot(act && nR + excl >= rs);
        if (over) {
          const int sl = __builtin_ctzll(over);
          stop_at = c + sl;
          cA += __popcll(nd & ((1ull << sl) - 1));
        } else {
          cA += __popcll(nd);
        }
      }
      if (stop_at >= 0 && i >= stop_at) kind = 3;
      uint32_t fp = 0;
      if (stop_at < 0) {
        const uint64_t m2 = __ballot(act && kind == 2);
        fp = (uint32_t)(nP + c2 + lanes_below(m2));
        if (act && kind == 2 && (int64_t)fp < W.pcap) {
          par[fp] = xchild<D>(par[pb + (i >> D)], (int)(i & (NK - 1)));
          pix[fp] = (uint32_t)(eb + i);   // the parent's own element, for the collapse below
        }
        c2 += __popcll(m2);
      }
      if (act) ek[eb + i] = ((uint32_t)kind << 30) | fp;
    }
    wave_mem_sync();
    nR += cA;
    Lmax = L;
    if (stop_at >= 0 || (c2 > 0 && L + 1 >= g)) {
      // the queued children are bottomed out: the level's overlapping elements become full intervals
      for (int64_t c = 0; c < K; c += 64) {
        const int64_t i = c + lane;
        if (i < K && (ek[eb + i] >> 30) == 2u) ek[eb + i] = 3u << 30;
      }
      // a sibling group wholly past the stop (all its elements bottomed out) chains into exactly its
      // parent's full interval: the parent becomes a kind-3 leaf and the group is dropped, so the
      // pre-merge list holds at most rangeStop + 2^D - 1 ranges
      if (stop_at >= 0 && L >= 2) {
        const int64_t keep = (stop_at + NK - 1) >> D;
        for (int64_t j = keep + lane; j < np; j += 64) ek[pix[pb + j]] = 3u << 30;
        if (lane == 0) lnp[L] = (int32_t)keep;
      }
      wave_mem_sync();
      break;
    }
    if (c2 == 0) break;
    if (nP + c2 > W.pcap || eb + K + (c2 << D) > W.ecap || L + 1 > XW_MAXL - 1) { err = QS_CAPACITY; break; }
    if (lane == 0) { lb[L + 1] = (int32_t)nP; le[L + 1] = (int32_t)(eb + K); lnp[L + 1] = (int32_t)c2; }
    wave_mem_sync();
    nP += c2;
    eb += K;
  }
  if (err) { finish(0, 0, err); return; }

  // ---- 2. order: subtree range counts (up), positions (down)
  auto S_of = [&](uint32_t x) -> uint32_t { return (x >> 30) == 2u ? tb[x & 0x3fffffffu] : (uint32_t)((x >> 30) != 0u); };
  for (int l = Lmax; l >= 1; --l) {
    const int64_t np = lnp[l], pb = lb[l], e0 = le[l];
    for (int64_t j = lane; j < np; j += 64) {
      uint32_t t = l == 1 ? 0u : 1u;
      for (int k = 0; k < NK; ++k) t += S_of(ek[e0 + j * NK + k]);
      tb[pb + j] = t;
    }
    wave_mem_sync();
  }
  const int64_t npre = tb[0];
  if (npre > W.rcap) { finish(0, 0, QS_CAPACITY); return; }
  if (lane == 0) tb[0] = 0;   // B of the unit element: its children start at 0
  wave_mem_sync();
  for (int l = 1; l <= Lmax; ++l) {
    const int64_t np = lnp[l], pb = lb[l], e0 = le[l];
    for (int64_t j = lane; j < np; j += 64) {
      uint32_t pos = tb[pb + j];
      const uint64_t pe = par[pb + j];
      for (int k = 0; k < NK; ++k) {
        const uint32_t x = ek[e0 + j * NK + k], kind = x >> 30;
        if (!kind) continue;
        const int64_t cs = xseq<D>(xchild<D>(pe, k), l, g);
        rlo[pos] = cs;
        rhi[pos] = kind == 2u ? cs : cs + xspan<D>(l, g);
        rcb[pos] = kind == 1u;
        if (kind == 2u) {
          const uint32_t t = tb[x & 0x3fffffffu];
          tb[x & 0x3fffffffu] = pos + 1;
          pos += t;
        } else {
          pos += 1;
        }
      }
    }
    wave_mem_sync();
  }

  // ---- 3. merge adjacent ranges (XZ2SFC.scala:231-249) into the batch buffer
  auto starts = [&](int64_t j) -> bool {   // range j opens a merged range
    return j == 0 || !(rlo[j] <= (int64_t)((uint64_t)rhi[j - 1] + 1u));
  };
  int64_t M = 0;
  for (int64_t c = 0; c < npre; c += 64) M += __popcll(__ballot(c + lane < npre && starts(c + lane)));
  unsigned long long obase = 0;
  if (lane == 0 && M > 0) obase = atomicAdd(a.bo.total, (unsigned long long)M);
  obase = __shfl(obase, 0, 64);
  int64_t runs = 0;          // merged ranges opened before this chunk
  bool carry_zero = false;   // the run continuing into this chunk has a range that is not contained
  for (int64_t c = 0; c < npre; c += 64) {
    const int64_t j = c + lane;
    const bool act = j < npre;
    const bool st = act && starts(j);
    const bool en = act && (j + 1 == npre || starts(j + 1));
    const uint64_t S = __ballot(st), Z = __ballot(act && !rcb[j]);
    const uint64_t le_mask = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1);
    const uint64_t sb = S & le_mask;   // starts at or below this lane
    bool zr;                           // a not-contained range in this lane's run up to here
    if (sb) {
      const int s0 = 63 - __builtin_clzll(sb);
      zr = (Z & le_mask & ~((1ull << s0) - 1)) != 0;
    } else {
      zr = carry_zero || (Z & le_mask) != 0;
    }
    const int64_t r = runs + __popcll(sb) - 1;
    if (st && (int64_t)obase + r < a.bo.dcap) a.bo.dbuf[obase + r].lower = rlo[j];
    if (en && (int64_t)obase + r < a.bo.dcap) {
      gm_range* o = &a.bo.dbuf[obase + r];
      o->upper = rhi[j];
      o->contained = zr ? 0 : 1;
      o->reserved = 0;
    }
    runs += __popcll(S);
    carry_zero = __shfl(zr, 63, 64);
  }
  finish((int64_t)obase, M, QS_OK);
}

// gather every query's ranges from the batch buffer into query order (one block per query)
__global__ __launch_bounds__(RTPB) void k_gather_ranges(const gm_range* __restrict__ buf, const int64_t* __restrict__ start,
                                                        const int64_t* __restrict__ off, int64_t nq,
                                                        gm_range* __restrict__ out) {
  for (int64_t q = blockIdx.x; q < nq; q += gridDim.x) {
    const int64_t a = off[q], n = off[q + 1] - a, s = start[q];
    for (int64_t j = threadIdx.x; j < n; j += RTPB) out[a + j] = buf[s + j];
  }
}

// ------------------------------------------------------------------ host driver

struct RangesJob {
  int kind;  // 2 = Z2, 3 = Z3, 12 = XZ2, 13 = XZ3
  int64_t nq;
  int range_stop;
};

inline int64_t next_pow2(int64_t v) { int64_t p = 1; while (p < v) p <<= 1; return p; }

}  // namespace gm

using namespace gm;

namespace {

template <class T>
int to_dev(gm_ctx* ctx, const T* h, size_t n, T** d) {
  GM_HIP(hipMallocAsync((void**)d, std::max<size_t>(n * sizeof(T), 16), ctx->stream));
  return copy_h2d(ctx, *d, h, n * sizeof(T));
}

// Shared driver.  Phase 1 runs every query with small workspaces (frontier / range lists of P1CAP,
// sorted in LDS), chunked only by a memory budget and launched back to back (the chunks reuse one
// stream-ordered workspace, no host round trip); the merged-range scratch aliases the frontier.
// Phase 2 re-runs the queries that overflowed it (status QS_CAPACITY) with the worst-case caps.
// Then the counts are scanned on the device, the batch buffer is gathered into query order and
// `finish` takes the result.  run_batch does this for queries [q_base, q_base + nq); the per-query
// arrays are indexed by absolute query id in the kernels (their base pointers are offset).
constexpr int64_t P1CAP = LDS_SORT;

// finish(total, dbuf, dstart, doff): query-order gather of the batch buffer and the copy out
template <class PerQFn, class LaunchFn, class FinishFn>
int run_batch(gm_ctx* ctx, int64_t q_base, int64_t nq, int64_t fcap, int64_t rcap, PerQFn& per_query, LaunchFn& launch,
              int64_t* out_off, int64_t cap, int64_t* needed, int32_t* query_status, FinishFn finish) {
  hipStream_t s = ctx->stream;
  rcap = next_pow2(std::max<int64_t>(rcap, 16));
  auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
  size_t free_b = 0, total_b = 0;
  int64_t budget = (int64_t)2 << 30;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
    budget = std::max<int64_t>(budget, std::min<int64_t>((int64_t)16 << 30, (int64_t)(free_b / 4)));
  // batch buffer: sized from the largest output seen on this context (at least 64 ranges a query),
  // bounded by the caller's capacity and the budget; a batch whose ranges overflow it but fit `cap`
  // runs once more with the exact size
  int64_t dcap = std::min<int64_t>(std::max<int64_t>({(int64_t)1 << 20, nq * 64, ctx->ranges_hint}),
                                   budget / (int64_t)sizeof(gm_range));
  dcap = std::max<int64_t>(1, std::min<int64_t>(cap, dcap));
  std::vector<int32_t> stats((size_t)nq);
  for (int attempt = 0;; ++attempt) {
    // batch arrays (scan workspace): buffer | start | offsets | count | status | qmap | scan partials | total
    gm_range* dbuf;
    int64_t *dstart, *doff, *dparts;
    int32_t *dcount, *dstatus, *dqmap;
    unsigned long long* dtotal;
    {
      const size_t sz[8] = {al((size_t)dcap * sizeof(gm_range)), al((size_t)nq * 8), al((size_t)(nq + 1) * 8),
                            al((size_t)nq * 4), al((size_t)nq * 4), al((size_t)nq * 4),
                            al((size_t)scan_partials_len(nq) * 8), 16};
      size_t tot = 0;
      for (size_t v : sz) tot += v;
      void* base = nullptr;
      int rc = ctx_workspace(ctx, WS_SCAN, tot, &base);
      if (rc) return rc;
      char* p = (char*)base;
      dbuf = (gm_range*)p; p += sz[0];
      dstart = (int64_t*)p; p += sz[1];
      doff = (int64_t*)p; p += sz[2];
      dcount = (int32_t*)p; p += sz[3];
      dstatus = (int32_t*)p; p += sz[4];
      dqmap = (int32_t*)p; p += sz[5];
      dparts = (int64_t*)p; p += sz[6];
      dtotal = (unsigned long long*)p;
    }
    GM_HIP(hipMemsetAsync(dtotal, 0, 8, s));
    // one pass over a query list with caps (fc, rc); qmap null = queries [q_base, q_base + count).  The
    // launcher's workspace is per_q(fc, rc) bytes per query, chunked by the memory budget
    auto pass = [&](int64_t count, const int32_t* qmap, int64_t fc, int64_t rc) -> int {
      const int64_t per_q = std::max<int64_t>(16, per_query(fc, rc));
      int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(count, budget / per_q));
      chunk = std::min<int64_t>(chunk, (int64_t)1 << 20);
      const int64_t m_max = std::min(chunk, count);
      void* base = nullptr;
      int wrc = ctx_workspace(ctx, WS_RANGES, (size_t)(m_max * per_q), &base);
      if (wrc) return wrc;
      for (int64_t q0 = 0; q0 < count; q0 += chunk) {
        const int64_t m = std::min(chunk, count - q0);
        // per-query arrays offset so that the kernels index them by absolute query id
        const BatchOut bo{qmap ? qmap + q0 : nullptr, 0, dbuf, dcap, dtotal, dstart - q_base, dcount - q_base,
                          dstatus - q_base};
        launch(qmap ? 0 : q_base + q0, m, fc, rc, (char*)base, bo);
        GM_CHECK_LAUNCH();
      }
      return GM_OK;
    };
    int rc = pass(nq, nullptr, std::min<int64_t>(fcap, P1CAP), std::min<int64_t>(rcap, P1CAP));
    if (rc) return rc;
    if (fcap > P1CAP || rcap > P1CAP) {
      rc = copy_d2h(ctx, stats.data(), dstatus, (size_t)nq * 4);
      if (rc) return rc;
      std::vector<int32_t> redo;
      for (int64_t i = 0; i < nq; ++i)
        if (stats[i] == QS_CAPACITY) redo.push_back((int32_t)(q_base + i));
      if (!redo.empty()) {
        rc = copy_h2d(ctx, dqmap, redo.data(), redo.size() * 4);
        if (!rc) rc = pass((int64_t)redo.size(), dqmap, fcap, rcap);
        if (rc) return rc;
      }
    }
    // device scan of the counts -> query-order offsets (total in out_off[nq])
    launch_excl_scan(s, dcount, nq, doff, dparts, doff + nq);
    GM_CHECK_LAUNCH();
    rc = copy_d2h(ctx, out_off, doff, (size_t)(nq + 1) * 8);
    if (!rc) rc = copy_d2h(ctx, stats.data(), dstatus, (size_t)nq * 4);
    if (rc) return rc;
    const int64_t total = out_off[nq];
    ctx->ranges_hint = std::max(ctx->ranges_hint, std::min(total, cap));
    if (total > dcap && total <= cap && attempt == 0) {
      dcap = total;
      continue;
    }
    if (query_status) memcpy(query_status, stats.data(), (size_t)nq * 4);
    if (needed) *needed = total;
    if (total > cap) return GM_E_CAPACITY;
    return total > 0 ? finish(total, dbuf, (const int64_t*)dstart, (const int64_t*)doff, nq) : GM_OK;
  }
}

// Batched ranges.  With pinned host output and enough queries, the queries run in chunks and chunk
// k's result copy (a second stream) overlaps chunk k + 1's kernels: the copy back of 10^7-10^8
// ranges costs as much as their computation.  The output is identical either way.
template <class PerQFn, class LaunchFn>
int run_ranges(gm_ctx* ctx, int64_t nq, int64_t fcap, int64_t rcap, PerQFn per_query, LaunchFn launch, int64_t* out_off,
               gm_range* out, int64_t cap, int64_t* needed, int32_t* query_status) {
  hipStream_t s = ctx->stream;
  int64_t qc = ctx->ranges_chunk > 0 ? ctx->ranges_chunk : (nq < 16384 ? nq : std::max<int64_t>(8192, (nq + 7) / 8));
  if (out && device_memory(out)) {   // device output (ranges consumed on the device): gathered in place
    return run_batch(ctx, 0, nq, fcap, rcap, per_query, launch, out_off, cap, needed, query_status,
                     [&](int64_t total, const gm_range* dbuf, const int64_t* dstart, const int64_t* doff, int64_t n) -> int {
                       hipLaunchKernelGGL(k_gather_ranges, dim3((unsigned)std::min<int64_t>(n, 65536)), dim3(RTPB), 0, s,
                                          dbuf, dstart, doff, n, out);
                       GM_CHECK_LAUNCH();
                       GM_HIP(hipStreamSynchronize(s));
                       return GM_OK;
                     });
  }
  if (qc >= nq || !out || !host_pinned(out)) {   // one batch: gather into scratch, one copy
    return run_batch(ctx, 0, nq, fcap, rcap, per_query, launch, out_off, cap, needed, query_status,
                     [&](int64_t total, const gm_range* dbuf, const int64_t* dstart, const int64_t* doff, int64_t n) -> int {
                       void* dout = nullptr;   // the range scratch is free again
                       int rc = ctx_workspace(ctx, WS_RANGES, (size_t)total * sizeof(gm_range), &dout);
                       if (rc) return rc;
                       hipLaunchKernelGGL(k_gather_ranges, dim3((unsigned)std::min<int64_t>(n, 65536)), dim3(RTPB), 0, s,
                                          dbuf, dstart, doff, n, (gm_range*)dout);
                       GM_CHECK_LAUNCH();
                       return copy_d2h(ctx, out, dout, (size_t)total * sizeof(gm_range));
                     });
  }
  int rc = ctx_copy_stream(ctx);
  if (rc) return rc;
  // two device result buffers, reused every other chunk once their copy is done (ev_copied)
  gm_range* dres[2] = {nullptr, nullptr};
  int64_t dres_cap[2] = {0, 0};
  bool used[2] = {false, false};
  auto release = [&]() {
    (void)hipStreamSynchronize(ctx->copy_stream);
    for (int k = 0; k < 2; ++k) if (dres[k]) (void)hipFree(dres[k]);
  };
  int64_t base = 0;
  bool over = false;
  int k = 0;
  std::vector<int64_t> off_c;
  for (int64_t c0 = 0; c0 < nq; c0 += qc, k ^= 1) {
    const int64_t m = std::min(qc, nq - c0);
    off_c.assign((size_t)m + 1, 0);
    int64_t tot = 0;
    rc = run_batch(ctx, c0, m, fcap, rcap, per_query, launch, off_c.data(), INT64_MAX / 32, &tot,
                   query_status ? query_status + c0 : nullptr,
                   [&](int64_t total, const gm_range* dbuf, const int64_t* dstart, const int64_t* doff, int64_t n) -> int {
                     if (over || base + total > cap) { over = true; return GM_OK; }   // capacity: counting only
                     if (used[k]) GM_HIP(hipStreamWaitEvent(s, ctx->ev_copied[k], 0));   // its last copy is done
                     if (dres_cap[k] < total) {
                       GM_HIP(hipStreamSynchronize(s));
                       if (dres[k]) (void)hipFree(dres[k]);
                       dres[k] = nullptr;
                       GM_HIP(hipMalloc(&dres[k], (size_t)total * sizeof(gm_range)));
                       dres_cap[k] = total;
                     }
                     hipLaunchKernelGGL(k_gather_ranges, dim3((unsigned)std::min<int64_t>(n, 65536)), dim3(RTPB), 0, s,
                                        dbuf, dstart, doff, n, dres[k]);
                     GM_CHECK_LAUNCH();
                     GM_HIP(hipEventRecord(ctx->ev_ready[k], s));
                     GM_HIP(hipStreamWaitEvent(ctx->copy_stream, ctx->ev_ready[k], 0));
                     GM_HIP(hipMemcpyAsync(out + base, dres[k], (size_t)total * sizeof(gm_range), hipMemcpyDeviceToHost,
                                           ctx->copy_stream));
                     GM_HIP(hipEventRecord(ctx->ev_copied[k], ctx->copy_stream));
                     used[k] = true;
                     return GM_OK;
                   });
    if (rc) { release(); return rc; }
    for (int64_t i = 0; i <= m; ++i) out_off[c0 + i] = base + off_c[(size_t)i];
    base += tot;
  }
  release();
  if (hipGetLastError() != hipSuccess) return hip_fail(hipErrorLaunchFailure, "batched ranges copy");
  if (needed) *needed = base;
  ctx->ranges_hint = std::max(ctx->ranges_hint, std::min(base, cap) / std::max<int64_t>(1, (nq + qc - 1) / qc));
  return base > cap ? GM_E_CAPACITY : GM_OK;
}

inline int stop_of(int max_ranges) { return max_ranges <= 0 ? INT32_MAX : max_ranges; }

// The Z kernel's workspace for m queries with caps (fc, rc): frontier ping / pong | rlo | rhi | rc |
// sort keys and ids (global-memory sort only) | merged scratch (unless it aliases the frontier)
struct ZLayout {
  bool lds_sort, alias;
  int64_t ocap, per_q;
};
inline ZLayout z_layout(int64_t fc, int64_t rc) {
  ZLayout z{};
  z.lds_sort = rc <= LDS_SORT;
  z.alias = 16 * fc >= rc * (int64_t)sizeof(gm_range);
  z.ocap = z.alias ? 16 * fc / (int64_t)sizeof(gm_range) : rc;
  z.per_q = 16 * fc + 17 * rc + (z.lds_sort ? 0 : 12 * rc) + (z.alias ? 0 : rc * (int64_t)sizeof(gm_range)) + 7 * 16;
  return z;
}
inline void z_place(char* base, int64_t m, int64_t fc, int64_t rc, ZRangesArgs& b) {
  const ZLayout z = z_layout(fc, rc);
  auto al = [](int64_t v) { return (v + 15) & ~(int64_t)15; };
  char* p = base;
  b.fa = (int64_t*)p; p += al(m * fc * 16);
  b.rlo = (int64_t*)p; p += al(m * rc * 8);
  b.rhi = (int64_t*)p; p += al(m * rc * 8);
  b.rc = (uint8_t*)p; p += al(m * rc);
  b.gkey = nullptr; b.gidx = nullptr;
  if (!z.lds_sort) { b.gkey = (int64_t*)p; p += al(m * rc * 8); b.gidx = (int32_t*)p; p += al(m * rc * 4); }
  b.out = z.alias ? (gm_range*)b.fa : (gm_range*)p;
  b.bo.ocap = z.ocap;
  b.fcap = fc; b.rcap = rc;
}

// workspace sizing: the FIFO never holds more than rangeStop + 2^D items before the budget fires
inline int64_t z_caps(int max_ranges, int D, int64_t cap_hint) {
  if (max_ranges > 0) return (int64_t)max_ranges + (1 << D) + 16;
  return std::max<int64_t>(cap_hint, 1 << 16);
}

// frees the stream-ordered input copies of one entry point on every return path
struct StreamFrees {
  hipStream_t s;
  void* p[4] = {nullptr, nullptr, nullptr, nullptr};
  explicit StreamFrees(hipStream_t st) : s(st) {}
  ~StreamFrees() {
    for (void* q : p)
      if (q) (void)hipFreeAsync(q, s);
  }
};

}  // namespace

extern "C" {

int gm_z3_ranges(gm_ctx* ctx, int64_t nq, const int32_t* box_off, const double* xy, const int32_t* time_off,
                 const int64_t* t, int period, int precision, int range_precision, int max_ranges, int max_recurse,
                 int64_t* out_off, gm_range* out, int64_t cap, int64_t* needed, int32_t* query_status) {
  if (!ctx || nq < 0 || !box_off || !time_off || !out_off || period < 0 || period > 3 || precision < 1 ||
      precision > 21 || range_precision < 1 || range_precision > 64)
    return GM_E_INVALID;
  if (nq == 0) { out_off[0] = 0; if (needed) *needed = 0; return GM_OK; }
  hipStream_t s = ctx->stream;
  const int64_t nbox = box_off[nq], ntim = time_off[nq];
  int32_t *dbo = nullptr, *dto = nullptr;
  double* dxy = nullptr;
  int64_t* dt = nullptr;
  StreamFrees fr(s);
  int rc = to_dev(ctx, box_off, (size_t)nq + 1, &dbo);
  fr.p[0] = dbo;
  if (!rc) { rc = to_dev(ctx, time_off, (size_t)nq + 1, &dto); fr.p[1] = dto; }
  if (!rc) { rc = to_dev(ctx, xy, (size_t)nbox * 4, &dxy); fr.p[2] = dxy; }
  if (!rc) { rc = to_dev(ctx, t, (size_t)ntim * 2, &dt); fr.p[3] = dt; }
  if (rc) return rc;
  ZRangesArgs a{};
  a.box_off = dbo; a.xy = dxy; a.time_off = dto; a.t = dt;
  a.lon = make_ndim(-180.0, 180.0, precision);
  a.lat = make_ndim(-90.0, 90.0, precision);
  a.tim = make_ndim(0.0, (double)max_offset(period), precision);
  a.range_precision = range_precision;
  a.range_stop = stop_of(max_ranges);
  a.recurse_stop = max_recurse < 0 ? INT32_MAX : max_recurse;   // Z3SFC.MaxRecursion = Int.MaxValue
  const int64_t zc = z_caps(max_ranges, 3, cap);
  rc = run_ranges(ctx, nq, zc, zc, [](int64_t fc, int64_t rcp) { return z_layout(fc, rcp).per_q; },
                  [&](int64_t q0, int64_t m, int64_t fc, int64_t rcp, char* base, const BatchOut& bo) {
                    ZRangesArgs b = a;
                    b.q0 = q0; b.bo = bo;
                    z_place(base, m, fc, rcp, b);
                    hipLaunchKernelGGL(k_zranges<3>, dim3((unsigned)m), dim3(RTPB), 0, s, b);
                  },
                  out_off, out, cap, needed, query_status);
  return rc;
}

int gm_z2_ranges(gm_ctx* ctx, int64_t nq, const int32_t* box_off, const double* xy, int precision,
                 int range_precision, int max_ranges, int max_recurse, int64_t* out_off, gm_range* out, int64_t cap,
                 int64_t* needed, int32_t* query_status) {
  if (!ctx || nq < 0 || !box_off || !out_off || precision < 1 || precision > 31 || range_precision < 1 ||
      range_precision > 64)
    return GM_E_INVALID;
  if (nq == 0) { out_off[0] = 0; if (needed) *needed = 0; return GM_OK; }
  hipStream_t s = ctx->stream;
  const int64_t nbox = box_off[nq];
  int32_t* dbo = nullptr;
  double* dxy = nullptr;
  StreamFrees fr(s);
  int rc = to_dev(ctx, box_off, (size_t)nq + 1, &dbo);
  fr.p[0] = dbo;
  if (!rc) { rc = to_dev(ctx, xy, (size_t)nbox * 4, &dxy); fr.p[1] = dxy; }
  if (rc) return rc;
  ZRangesArgs a{};
  a.box_off = dbo; a.xy = dxy; a.time_off = nullptr; a.t = nullptr;
  a.lon = make_ndim(-180.0, 180.0, precision);
  a.lat = make_ndim(-90.0, 90.0, precision);
  a.range_precision = range_precision;
  a.range_stop = stop_of(max_ranges);
  a.recurse_stop = max_recurse < 0 ? 7 : max_recurse;   // ZN.DefaultRecurse (ZN.scala:293)
  const int64_t zc = z_caps(max_ranges, 2, cap);
  rc = run_ranges(ctx, nq, zc, zc, [](int64_t fc, int64_t rcp) { return z_layout(fc, rcp).per_q; },
                  [&](int64_t q0, int64_t m, int64_t fc, int64_t rcp, char* base, const BatchOut& bo) {
                    ZRangesArgs b = a;
                    b.q0 = q0; b.bo = bo;
                    z_place(base, m, fc, rcp, b);
                    hipLaunchKernelGGL(k_zranges<2>, dim3((unsigned)m), dim3(RTPB), 0, s, b);
                  },
                  out_off, out, cap, needed, query_status);
  return rc;
}

static int xz_ranges(gm_ctx* ctx, int D, int64_t nq, const int32_t* win_off, const double* windows, int g,
                     int period, int max_ranges, int64_t* out_off, gm_range* out, int64_t cap, int64_t* needed,
                     int32_t* query_status) {
  if (!ctx || nq < 0 || !win_off || !out_off || g < 1 || g > (D == 2 ? 29 : 19) || period < 0 || period > 3)
    return GM_E_INVALID;
  if (nq == 0) { out_off[0] = 0; if (needed) *needed = 0; return GM_OK; }
  hipStream_t s = ctx->stream;
  const int64_t nw = win_off[nq];
  int32_t* dwo = nullptr;
  double* dw = nullptr;
  StreamFrees fr(s);
  int rc = to_dev(ctx, win_off, (size_t)nq + 1, &dwo);
  fr.p[0] = dwo;
  if (!rc) { rc = to_dev(ctx, windows, (size_t)nw * 2 * D, &dw); fr.p[1] = dw; }
  if (rc) return rc;
  XZWaveArgs a{};
  a.win_off = dwo; a.win = dw; a.g = g; a.zhi = (double)max_offset(period);
  a.range_stop = stop_of(max_ranges);
  // the walk processes at most rangeStop non-disjoint elements, each at most one parent of the next
  // level; the pre-merge list holds those ranges plus the unprocessed rest of one sibling group
  int64_t fcap, rcap;
  if (max_ranges > 0) {
    // a budget past the unbounded caps (a caller passing a huge maxRanges to mean "unlimited") gets
    // the unbounded caps, so a query past them reports QS_CAPACITY like an unbounded one
    fcap = std::min<int64_t>((int64_t)max_ranges + 2, (int64_t)1 << 24);
    rcap = std::min<int64_t>((int64_t)max_ranges + (1 << D) + 16, fcap << (D + 1));
  } else {
    // unbounded (maxRanges <= 0): the frontier is not bounded by a budget, so the worst-case caps are
    // capped instead (~320 B per frontier slot per query for XZ3) -- a query past them reports
    // QS_CAPACITY in its status -- and kept inside the kernel's packed fields: parent ids in 30 bits of
    // an element word, element / range counts in int32
    fcap = std::min<int64_t>(std::max<int64_t>(cap, 1 << 16), (int64_t)1 << 24);
    rcap = (int64_t)fcap << (D + 1);
  }
  if (fcap >= ((int64_t)1 << 30) || (fcap << D) >= ((int64_t)1 << 31) || rcap >= ((int64_t)1 << 31))
    return hip_fail(hipErrorInvalidValue, "xz ranges: workspace caps past the kernel's packed fields");
  rc = run_ranges(ctx, nq, fcap, rcap, [D](int64_t fc, int64_t rcp) { return xz_ws(D, fc, rcp).stride; },
                  [&](int64_t q0, int64_t m, int64_t fc, int64_t rcp, char* base, const BatchOut& bo) {
                    XZWaveArgs b = a;
                    b.q0 = q0; b.m = m; b.bo = bo; b.base = base;
                    b.ws = xz_ws(D, fc, rcp);
                    const unsigned grid = (unsigned)((m + XW_TPB / 64 - 1) / (XW_TPB / 64));
                    if (D == 2) hipLaunchKernelGGL(k_xzranges_w<2>, dim3(grid), dim3(XW_TPB), 0, s, b);
                    else hipLaunchKernelGGL(k_xzranges_w<3>, dim3(grid), dim3(XW_TPB), 0, s, b);
                  },
                  out_off, out, cap, needed, query_status);
  return rc;
}

int gm_zranges(gm_ctx* ctx, int dims, int64_t nq, const int32_t* bound_off, const int64_t* zbounds,
               int range_precision, int max_ranges, int max_recurse, int64_t* out_off, gm_range* out, int64_t cap,
               int64_t* needed, int32_t* query_status) {
  if (!ctx || (dims != 2 && dims != 3) || nq < 0 || !bound_off || !out_off || range_precision < 1 ||
      range_precision > 64)
    return GM_E_INVALID;
  if (nq == 0) { out_off[0] = 0; if (needed) *needed = 0; return GM_OK; }
  hipStream_t s = ctx->stream;
  const int64_t nb = bound_off[nq];
  if (nb > 0 && !zbounds) return GM_E_INVALID;
  int32_t* dbo = nullptr;
  int64_t* dzb = nullptr;
  StreamFrees fr(s);
  int rc = to_dev(ctx, bound_off, (size_t)nq + 1, &dbo);
  fr.p[0] = dbo;
  if (!rc) { rc = to_dev(ctx, zbounds, (size_t)nb * 2, &dzb); fr.p[1] = dzb; }
  if (rc) return rc;
  ZRangesArgs a{};
  a.zb_off = dbo; a.zb = dzb;
  a.range_precision = range_precision;
  a.range_stop = stop_of(max_ranges);
  a.recurse_stop = max_recurse < 0 ? 7 : max_recurse;   // maxRecurse = Some(ZN.DefaultRecurse) (ZN.scala:113,293)
  const int64_t zc = z_caps(max_ranges, dims, cap);
  rc = run_ranges(ctx, nq, zc, zc, [](int64_t fc, int64_t rcp) { return z_layout(fc, rcp).per_q; },
                  [&](int64_t q0, int64_t m, int64_t fc, int64_t rcp, char* base, const BatchOut& bo) {
                    ZRangesArgs b = a;
                    b.q0 = q0; b.bo = bo;
                    z_place(base, m, fc, rcp, b);
                    if (dims == 3) hipLaunchKernelGGL(k_zranges<3>, dim3((unsigned)m), dim3(RTPB), 0, s, b);
                    else hipLaunchKernelGGL(k_zranges<2>, dim3((unsigned)m), dim3(RTPB), 0, s, b);
                  },
                  out_off, out, cap, needed, query_status);
  return rc;
}

int gm_xz2_ranges(gm_ctx* ctx, int64_t nq, const int32_t* win_off, const double* windows, int g, int max_ranges,
                  int64_t* out_off, gm_range* out, int64_t cap, int64_t* needed, int32_t* query_status) {
  return xz_ranges(ctx, 2, nq, win_off, windows, g, GM_WEEK, max_ranges, out_off, out, cap, needed, query_status);
}

int gm_xz3_ranges(gm_ctx* ctx, int64_t nq, const int32_t* win_off, const double* windows, int g, int period,
                  int max_ranges, int64_t* out_off, gm_range* out, int64_t cap, int64_t* needed,
                  int32_t* query_status) {
  return xz_ranges(ctx, 3, nq, win_off, windows, g, period, max_ranges, out_off, out, cap, needed, query_status);
}

}  // extern "C"
