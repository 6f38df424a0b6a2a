// gm_filter.hip -- fused key-space / strict filter scans with wave-ballot compaction.
//
// Z3Filter.inBounds (idx/filters/Z3Filter.scala:26-62) is evaluated for every row of a columnar
// key store in one pass: 10 B/row (bin i16 + z i64) in, 1 bit/row out.  The Scala code runs it per
// row inside RowFilterIterator (geomesa-accumulo-iterators/.../RowFilterIterator.scala:52-66) or
// Z3HBaseFilter; here a wave of 64 rows produces one 64-bit ballot word.
//
// Output pipeline (all on the context stream, deterministic, ids ascending):
//   pass A  k_*_mask     : per-row predicate -> mask words + per-block match counts
//   pass B  launch_excl_scan (gm_scan.hpp): exclusive scan of the per-block counts
//   pass C  k_mask_to_ids: expand mask bits into row ids at the scanned offsets
// Pass C reads n/8 bytes of mask, so the ids cost ~1/80 of pass A's traffic plus 8 B per match.
#include <string.h>

#include <algorithm>
#include <vector>

#include "gm_scan.hpp"

namespace gm {

// ------------------------------------------------------------------ device filter descriptor
// flat int32 layout (built on the host from Z3Filter.serializeToBytes):
//   [0] nxy, [1] min_epoch, [2] max_epoch, [3] nt, [4] reserved
//   [5 .. 5+4*nxy)        xy boxes (xmin, ymin, xmax, ymax) in normalized cells
//   then nt (start, end) interval index pairs, (-1, -1) for a null epoch
//   then the intervals (t0, t1)
__device__ __forceinline__ bool z3_in_bounds_time(const int32_t* f, int16_t epoch, int64_t z);

// Z3Filter.pointInBounds && timeInBounds (Z3Filter.scala:31-62)
__device__ __forceinline__ bool z3_in_bounds(const int32_t* f, int16_t epoch, int64_t z) {
  const int nxy = f[0];
  const int32_t* xy = f + 5;
  const int32_t x = z3_combine(z), y = z3_combine(z >> 1);
  bool pin = false;
  for (int i = 0; i < nxy; ++i) {
    const int32_t* q = xy + 4 * i;
    if (x >= q[0] && x <= q[2] && y >= q[1] && y <= q[3]) { pin = true; break; }
  }
  if (!pin) return false;
  return z3_in_bounds_time(f, epoch, z);
}

// timeInBounds part of Z3Filter.inBounds (Z3Filter.scala:45-62)
__device__ __forceinline__ bool z3_in_bounds_time(const int32_t* f, int16_t epoch, int64_t z) {
  const int nxy = f[0];
  const int32_t* xy = f + 5;
  const int min_e = f[1], max_e = f[2];
  if (epoch > max_e || epoch < min_e) return true;   // whole epochs are left out (:46-47)
  const int nt = f[3];
  const int32_t* ep = xy + 4 * nxy;
  const int k = epoch - min_e;
  if (k >= nt) return true;
  const int a = ep[2 * k], b = ep[2 * k + 1];
  if (a < 0) return true;                             // null epoch -> true (:49)
  const int32_t* tiv = ep + 2 * nt;
  const int32_t t = z3_combine(z >> 2);
  for (int i = a; i < b; ++i)
    if (t >= tiv[2 * i] && t <= tiv[2 * i + 1]) return true;
  return false;
}

__device__ __forceinline__ bool bin_allowed(const int32_t* br, int nbr, int16_t b) {
  if (nbr == 0) return true;
  for (int i = 0; i < nbr; ++i)
    if (b >= br[2 * i] && b <= br[2 * i + 1]) return true;
  return false;
}

// block-level match count from per-wave popcounts
__device__ __forceinline__ void block_count(int local, int32_t* block_counts) {
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(&s_cnt, local);
  __syncthreads();
  if (threadIdx.x == 0) block_counts[blockIdx.x] = s_cnt;
}

// pass A for Z3Filter: filter descriptor staged in LDS once per block
__global__ __launch_bounds__(FTPB) void k_z3filter_mask(const int16_t* __restrict__ bin, const int64_t* __restrict__ z,
                                                        int64_t n, const int32_t* __restrict__ fdesc, int fwords,
                                                        const int32_t* __restrict__ bins, int nbr,
                                                        uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  extern __shared__ int32_t s_f[];
  for (int i = threadIdx.x; i < fwords; i += FTPB) s_f[i] = fdesc[i];
  int32_t* s_bins = s_f + fwords;
  for (int i = threadIdx.x; i < 2 * nbr; i += FTPB) s_bins[i] = bins[i];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * FROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int local = 0;
#pragma unroll 4
  for (int u = 0; u < FELEMS; ++u) {
    const int64_t i = base + (int64_t)u * FTPB + threadIdx.x;
    bool ok = false;
    if (i < n) {
      const int16_t b = bin[i];
      const int64_t zz = z[i];
      ok = bin_allowed(s_bins, nbr, b) && z3_in_bounds(s_f, b, zz);
    }
    const uint64_t w = __ballot(ok);
    if (lane == 0) {
      const int64_t word = (base + (int64_t)u * FTPB + wave * 64) >> 6;
      if ((word << 6) < n) mask[word] = w;
      local += __popcll(w);
    }
  }
  block_count(local, block_counts);
}

// Z2Filter.inBounds (idx/filters/Z2Filter.scala:20-35)
__global__ __launch_bounds__(FTPB) void k_z2filter_mask(const int64_t* __restrict__ z, int64_t n,
                                                        const int32_t* __restrict__ xy, int nxy,
                                                        uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  extern __shared__ int32_t s_xy[];
  for (int i = threadIdx.x; i < 4 * nxy; i += FTPB) s_xy[i] = xy[i];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * FROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int local = 0;
#pragma unroll 4
  for (int u = 0; u < FELEMS; ++u) {
    const int64_t i = base + (int64_t)u * FTPB + threadIdx.x;
    bool ok = false;
    if (i < n) {
      const int64_t zz = z[i];
      const int32_t x = z2_combine(zz), y = z2_combine(zz >> 1);
      for (int k = 0; k < nxy; ++k) {
        const int32_t* q = s_xy + 4 * k;
        if (x >= q[0] && x <= q[2] && y >= q[1] && y <= q[3]) { ok = true; break; }
      }
    }
    const uint64_t w = __ballot(ok);
    if (lane == 0) {
      const int64_t word = (base + (int64_t)u * FTPB + wave * 64) >> 6;
      if ((word << 6) < n) mask[word] = w;
      local += __popcll(w);
    }
  }
  block_count(local, block_counts);
}

// strict: GeoTools BBOX on a point (inclusive) AND FastDuring (exclusive, ms)
template <bool DURING>
__global__ __launch_bounds__(FTPB) void k_strict_mask(const double* __restrict__ x, const double* __restrict__ y,
                                                      const int64_t* __restrict__ t, int64_t n, double bx0, double by0,
                                                      double bx1, double by1, int64_t lo, int64_t hi,
                                                      uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  const int64_t base = (int64_t)blockIdx.x * FROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int local = 0;
#pragma unroll 4
  for (int u = 0; u < FELEMS; ++u) {
    const int64_t i = base + (int64_t)u * FTPB + threadIdx.x;
    bool ok = false;
    if (i < n) {
      const double px = x[i], py = y[i];
      ok = px >= bx0 && px <= bx1 && py >= by0 && py <= by1;
      if (DURING) {
        const int64_t tt = t[i];
        ok = ok && tt > lo && tt < hi;
      }
    }
    const uint64_t w = __ballot(ok);
    if (lane == 0) {
      const int64_t word = (base + (int64_t)u * FTPB + wave * 64) >> 6;
      if ((word << 6) < n) mask[word] = w;
      local += __popcll(w);
    }
  }
  block_count(local, block_counts);
}

// Descriptor access.  Per-row reads of even wave-uniform descriptor words cost scalar loads plus
// loop and exec-mask bookkeeping, and decoding x and y with Z3.combine costs ~60 VALU per row
// (PMC: ~110 VALU per row, issue-bound at 45% of HBM).  The fast path (<= FBOX boxes,
// <= FBIN bin ranges: every bbox/during query) instead keeps the boxes as DILATED bounds in
// registers: spreading bits to every third position preserves order, so
//     lo <= Z3.combine(z) <= hi   <=>   dilate(lo) <= (z & X_BITS) <= dilate(hi)     (unsigned)
// (and likewise for y with the mask shifted by one).  A row then costs two ANDs and four 64-bit
// compares per box.  Bounds outside the 21-bit dimension are clamped on the host (an empty box gets
// lo > hi).  Only rows that pass bin + box read the per-epoch interval table (lane-varying, L1/L2).
constexpr int FBOX = 4, FBIN = 4;
constexpr uint64_t Z3_XBITS = 0x1249249249249249ull;   // Z3.combine's mask (Z3.scala:84)

// bin_allowed && Z3Filter.inBounds with dilated boxes and bin ranges in registers
__device__ __forceinline__ bool z3_row_fast(const uint64_t* bx, int nxy, const int32_t* br, int nbr,
                                            const int32_t* __restrict__ fdesc, int16_t b, int64_t z) {
  bool ba = nbr == 0;
#pragma unroll
  for (int i = 0; i < FBIN; ++i) {
    if (i >= nbr) break;
    ba |= (b >= br[2 * i]) & (b <= br[2 * i + 1]);
  }
  const uint64_t xv = (uint64_t)z & Z3_XBITS, yv = (uint64_t)z & (Z3_XBITS << 1);
  bool pin = false;
#pragma unroll
  for (int i = 0; i < FBOX; ++i) {
    if (i >= nxy) break;
    pin |= (xv >= bx[4 * i]) & (xv <= bx[4 * i + 1]) & (yv >= bx[4 * i + 2]) & (yv <= bx[4 * i + 3]);
  }
  if (!(ba && pin)) return false;
  return z3_in_bounds_time(fdesc, b, z);
}

// The generic path reads the descriptor straight from global memory with wave-uniform indices.
template <bool FAST>
__global__ __launch_bounds__(FTPB) void k_z3filter_mask_v(const sv2* __restrict__ bin2, const lv2* __restrict__ z2,
                                                          int64_t n, const uint64_t* __restrict__ dil,
                                                          const int32_t* __restrict__ fdesc,
                                                          const int32_t* __restrict__ bins, int nbr,
                                                          uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  sv2 bv[FPAIRS];
  lv2 zv[FPAIRS];
  const int nxy = fdesc[0];
  uint64_t bx[4 * FBOX];
  int32_t br[2 * FBIN];
#pragma unroll
  for (int i = 0; i < 4 * FBOX; ++i) bx[i] = (FAST && i < 4 * nxy) ? dil[i] : 0;
#pragma unroll
  for (int i = 0; i < 2 * FBIN; ++i) br[i] = (FAST && i < 2 * nbr) ? bins[i] : 0;
  auto pred = [&](int16_t b, int64_t z) {
    if (FAST) return z3_row_fast(bx, nxy, br, nbr, fdesc, b, z);
    return bin_allowed(bins, nbr, b) && z3_in_bounds(fdesc, b, z);
  };
  pair_scan(
      n, mask, block_counts,
      [&](int64_t p, int u) { bv[u] = __builtin_nontemporal_load(&bin2[p]); zv[u] = __builtin_nontemporal_load(&z2[p]); },
      [&](int u, int j) { return j ? pred(bv[u].y, zv[u].y) : pred(bv[u].x, zv[u].x); },
      [&](int64_t p) { return pred(((const int16_t*)bin2)[2 * p], ((const int64_t*)z2)[2 * p]); });
}

__device__ __forceinline__ bool z2_in_xy(const int32_t* __restrict__ xy, int nxy, int64_t zz) {
  const int32_t x = z2_combine(zz), y = z2_combine(zz >> 1);
  for (int k = 0; k < nxy; ++k) {
    const int32_t* q = xy + 4 * k;
    if (x >= q[0] && x <= q[2] && y >= q[1] && y <= q[3]) return true;
  }
  return false;
}

// Z2: Z2.combine yields 32 bits (z bit 62 -> x bit 31, the sign bit of z -> y bit 31) compared as
// signed Ints, so the dilated form flips the dimension's top bit (signed -> unsigned order) on both
// sides: lo <= x  <=>  dilate(lo ^ 2^31) <= (z & X_BITS) ^ top.
constexpr uint64_t Z2_XBITS = 0x5555555555555555ull;

template <bool FAST>
__global__ __launch_bounds__(FTPB) void k_z2filter_mask_v(const lv2* __restrict__ z2, int64_t n,
                                                          const uint64_t* __restrict__ dil,
                                                          const int32_t* __restrict__ xy, int nxy,
                                                          uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  lv2 zv[FPAIRS];
  uint64_t bx[4 * FBOX];
#pragma unroll
  for (int i = 0; i < 4 * FBOX; ++i) bx[i] = (FAST && i < 4 * nxy) ? dil[i] : 0;
  auto pred = [&](int64_t zz) {
    if (!FAST) return z2_in_xy(xy, nxy, zz);
    const uint64_t xv = ((uint64_t)zz & Z2_XBITS) ^ (1ull << 62), yv = ((uint64_t)zz & (Z2_XBITS << 1)) ^ (1ull << 63);
    bool pin = false;
#pragma unroll
    for (int i = 0; i < FBOX; ++i) {
      if (i >= nxy) break;
      pin |= (xv >= bx[4 * i]) & (xv <= bx[4 * i + 1]) & (yv >= bx[4 * i + 2]) & (yv <= bx[4 * i + 3]);
    }
    return pin;
  };
  pair_scan(
      n, mask, block_counts, [&](int64_t p, int u) { zv[u] = __builtin_nontemporal_load(&z2[p]); },
      [&](int u, int j) { return pred(j ? zv[u].y : zv[u].x); },
      [&](int64_t p) { return pred(((const int64_t*)z2)[2 * p]); });
}

template <bool DURING>
__global__ __launch_bounds__(FTPB) void k_strict_mask_v(const dv2* __restrict__ x, const dv2* __restrict__ y,
                                                        const lv2* __restrict__ t, int64_t n, double bx0, double by0,
                                                        double bx1, double by1, int64_t lo, int64_t hi,
                                                        uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts) {
  auto pred = [&](double px, double py, int64_t tt) {
    bool ok = px >= bx0 && px <= bx1 && py >= by0 && py <= by1;
    if (DURING) ok = ok && tt > lo && tt < hi;
    return ok;
  };
  dv2 xv[FPAIRS], yv[FPAIRS];
  lv2 tv[FPAIRS];
  pair_scan(
      n, mask, block_counts,
      [&](int64_t p, int u) {
        xv[u] = __builtin_nontemporal_load(&x[p]);
        yv[u] = __builtin_nontemporal_load(&y[p]);
        if (DURING) tv[u] = __builtin_nontemporal_load(&t[p]);
        else tv[u] = lv2{0, 0};
      },
      [&](int u, int j) { return j ? pred(xv[u].y, yv[u].y, tv[u].y) : pred(xv[u].x, yv[u].x, tv[u].x); },
      [&](int64_t p) {
        return pred(((const double*)x)[2 * p], ((const double*)y)[2 * p], DURING ? ((const int64_t*)t)[2 * p] : 0);
      });
}

// pass C: one block per pass-A block; per (step, wave) popcount prefix gives each lane its slot
__global__ __launch_bounds__(FTPB) void k_mask_to_ids(const uint64_t* __restrict__ mask, int64_t n,
                                                      const int64_t* __restrict__ offsets, int64_t* __restrict__ ids,
                                                      int64_t cap) {
  __shared__ int32_t s_pre[FELEMS * (FTPB / 64)];
  const int64_t base = (int64_t)blockIdx.x * FROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NW = FTPB / 64;
  if (threadIdx.x < FELEMS * NW) {
    const int u = threadIdx.x / NW, w = threadIdx.x % NW;
    const int64_t word = (base + (int64_t)u * FTPB + w * 64) >> 6;
    s_pre[threadIdx.x] = ((word << 6) < n) ? __popcll(mask[word]) : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int k = 0; k < FELEMS * NW; ++k) { int c = s_pre[k]; s_pre[k] = run; run += c; }
  }
  __syncthreads();
  const int64_t blk_off = offsets[blockIdx.x];
  for (int u = 0; u < FELEMS; ++u) {
    const int64_t word = (base + (int64_t)u * FTPB + wave * 64) >> 6;
    if ((word << 6) >= n) break;
    const uint64_t w = mask[word];
    if ((w >> lane) & 1ull) {
      const int before = __popcll(w & ((1ull << lane) - 1ull));
      const int64_t slot = blk_off + s_pre[u * NW + wave] + before;
      if (slot < cap) ids[slot] = (word << 6) + lane;
    }
  }
}

// ------------------------------------------------------------------ row-key bytes (RowFilter.inBounds)
// RowFilterIterator.findTop calls filter.inBounds(row bytes, offset) once per row
// (geomesa-accumulo-iterators/.../RowFilterIterator.scala:52-66).  Here row i is
// rows[row_off[i] .. row_off[i+1]): the key is read from aligned dwords covering its bytes (a dword
// holding at least one byte of the row never crosses a page) and byte-swapped from big-endian
// (ByteArrays.readShort / readLong).  A row too short for its key is a non-match counted in
// *short_rows (the JVM read would throw ArrayIndexOutOfBoundsException).
template <int KEYLEN>
__device__ __forceinline__ bool row_key(const uint8_t* __restrict__ rows, const int64_t* __restrict__ row_off,
                                        int64_t i, int key_offset, int16_t& epoch, int64_t& z) {
  const int64_t a = row_off[i], len = row_off[i + 1] - a;
  if (len < (int64_t)key_offset + KEYLEN) return false;
  const uintptr_t p = (uintptr_t)(rows + a + key_offset);
  const uint32_t* w = (const uint32_t*)(p & ~(uintptr_t)3);
  const int sh = (int)(p & 3);
  const uint32_t w0 = w[0], w1 = w[1];
  const uint32_t w2 = (KEYLEN == 10 || sh > 0) ? w[2] : 0u;
  const uint32_t w3 = (KEYLEN == 10 && sh == 3) ? w[3] : 0u;
  const uint64_t lo = (uint64_t)w0 | ((uint64_t)w1 << 32), hi = (uint64_t)w2 | ((uint64_t)w3 << 32);
  const uint64_t k0 = sh ? (lo >> (8 * sh)) | (hi << (64 - 8 * sh)) : lo;   // key bytes 0..7, little-endian
  if (KEYLEN == 8) {
    z = (int64_t)__builtin_bswap64(k0);
    epoch = 0;
  } else {
    const uint64_t k1 = hi >> (8 * sh);                                      // key bytes 8..
    epoch = (int16_t)(uint16_t)(((k0 & 0xffu) << 8) | ((k0 >> 8) & 0xffu));
    z = (int64_t)__builtin_bswap64((k0 >> 16) | (k1 << 48));
  }
  return true;
}

template <bool Z3>
__global__ __launch_bounds__(FTPB) void k_filter_rows_mask(const uint8_t* __restrict__ rows,
                                                           const int64_t* __restrict__ row_off, int key_offset,
                                                           int64_t n, const int32_t* __restrict__ fdesc, int fwords,
                                                           uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts,
                                                           unsigned long long* __restrict__ short_rows) {
  extern __shared__ int32_t s_f[];
  for (int i = threadIdx.x; i < fwords; i += FTPB) s_f[i] = fdesc[i];
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * FROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int local = 0, nshort = 0;
  for (int u = 0; u < FELEMS; ++u) {
    const int64_t i = base + (int64_t)u * FTPB + threadIdx.x;
    bool ok = false;
    if (i < n) {
      int16_t e;
      int64_t zz;
      if (row_key<Z3 ? 10 : 8>(rows, row_off, i, key_offset, e, zz)) {
        ok = Z3 ? z3_in_bounds(s_f, e, zz) : z2_in_xy(s_f, fwords / 4, zz);   // Z3Filter.scala:26-28 / Z2Filter
      } else {
        ++nshort;
      }
    }
    const uint64_t w = __ballot(ok);
    if (lane == 0) {
      const int64_t word = (base + (int64_t)u * FTPB + wave * 64) >> 6;
      if ((word << 6) < n) mask[word] = w;
      local += __popcll(w);
    }
  }
  if (nshort && short_rows) atomicAdd(short_rows, (unsigned long long)nshort);
  block_count(local, block_counts);
}

// ------------------------------------------------------------------ range scan of a sorted table
// gm_key_range_scan: the seek-and-filter loop of a Z3 query against a table sorted by gm_sort_keys.
// Each range [lo, hi] of the (shard, bin, z) key prefix (getRangeBytes, Z3IndexKeySpace.scala:196-238)
// maps to a row interval by two binary searches; the intervals' rows are the candidates
// (Accumulo/HBase scan), and Z3Filter.inBounds runs on each (RowFilterIterator.scala:52-66) in the
// same mask -> block scan -> ordered compaction pipeline as the full scans.
struct DevRange {
  uint64_t z_lo, z_hi;
  uint32_t kb_lo, kb_hi;   // shard << 16 | (uint16) bin
};

__device__ __forceinline__ bool key_lt(uint32_t ka, uint64_t za, uint32_t kb, uint64_t zb) {
  return ka < kb || (ka == kb && za < zb);
}

// bin = null: a key space without a time bin (Z2 / XZ2: [shard][z BE64]), every row's bin reads as 0
__device__ __forceinline__ uint32_t row_kb(const uint8_t* sh, const uint16_t* bin, int64_t i) {
  return ((uint32_t)(sh ? sh[i] : 0) << 16) | (bin ? bin[i] : 0u);
}

// row interval of each range: [first row >= lo, first row > hi)
__global__ __launch_bounds__(FTPB) void k_range_bounds(const uint8_t* __restrict__ sh, const uint16_t* __restrict__ bin,
                                                       const uint64_t* __restrict__ z, int64_t n,
                                                       const DevRange* __restrict__ rg, int64_t nr,
                                                       int64_t* __restrict__ start, int64_t* __restrict__ len) {
  const int64_t r = (int64_t)blockIdx.x * FTPB + threadIdx.x;
  if (r >= nr) return;
  const DevRange q = rg[r];
  int64_t lo = 0, hi = n;  // lower_bound(lo key)
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (key_lt(row_kb(sh, bin, m), z[m], q.kb_lo, q.z_lo)) lo = m + 1; else hi = m;
  }
  const int64_t a = lo;
  hi = n;  // upper_bound(hi key)
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (!key_lt(q.kb_hi, q.z_hi, row_kb(sh, bin, m), z[m])) lo = m + 1; else hi = m;
  }
  start[r] = a;
  len[r] = lo - a;
}

// in-place exclusive scan of int64 lengths (one block); total -> a[len]
__global__ __launch_bounds__(1024) void k_scan_i64(int64_t* __restrict__ a, int64_t len) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (len + 1023) / 1024, lo = t * per, hi = min(len, lo + per);
  int64_t s = 0;
  for (int64_t k = lo; k < hi; ++k) s += a[k];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int64_t k = lo; k < hi; ++k) { const int64_t c = a[k]; a[k] = run; run += c; }
  if (t == 1023) a[len] = part[1023];
}

// candidate c -> its range (upper_bound over the scanned offsets, minus one) -> table row
__device__ __forceinline__ int64_t cand_row(const int64_t* __restrict__ coff, const int64_t* __restrict__ start,
                                            int64_t nr, int64_t c) {
  int64_t lo = 0, hi = nr;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (coff[m] <= c) lo = m + 1; else hi = m;
  }
  const int64_t r = lo - 1;
  return start[r] + (c - coff[r]);
}


// candidate-space mask: candidate c = the c-th row inside the (disjoint, sorted) intervals.  RF: the row
// filter the tablet server runs on the key (RowFilterIterator.scala:52-66): none, Z3Filter.inBounds on
// (bin, z) (Z3Filter.scala:26-62) or Z2Filter.inBounds on z (Z2Filter.scala:20-35).  ENV / DUR: the full
// filter on the feature (the XZ key spaces' useFullFilter = true, XZ2IndexKeySpace.scala:122-125,
// XZ3IndexKeySpace.scala:247-250) over the caller's input-order columns, reached through perm: JTS
// Envelope.intersects with any query box (inclusive), and FastDuring (exclusive, ms) on the dtg.
enum : int { RF_NONE = 0, RF_Z3 = 1, RF_Z2 = 2 };
struct FullFilter {
  const double *xmin, *ymin, *xmax, *ymax;   // feature envelopes (input order)
  const int64_t* t;                           // feature dtg (input order)
  const double* boxes;                        // nbox x (xmin, ymin, xmax, ymax), device
  int nbox;
  int64_t t_lo, t_hi;
  const int64_t* perm;                        // table row -> input row (null: the identity)
};
// JTS Envelope.intersects(Envelope): false for a null envelope (maxx < minx) on either side
__device__ __forceinline__ bool env_intersects(double ax0, double ay0, double ax1, double ay1, const double* q) {
  if (ax1 < ax0 || q[2] < q[0]) return false;
  return !(q[0] > ax1 || q[2] < ax0 || q[1] > ay1 || q[3] < ay0);
}
template <int RF, bool ENV, bool DUR>
__global__ __launch_bounds__(FTPB) void k_range_mask(const uint16_t* __restrict__ bin, const uint64_t* __restrict__ z,
                                                     const int64_t* __restrict__ coff, const int64_t* __restrict__ start,
                                                     int64_t nr, int64_t total, const int32_t* __restrict__ fdesc, int nxy,
                                                     FullFilter ff, uint64_t* __restrict__ mask,
                                                     int32_t* __restrict__ block_counts) {
  const int64_t base = (int64_t)blockIdx.x * FROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int local = 0;
  for (int u = 0; u < FELEMS; ++u) {
    const int64_t c = base + (int64_t)u * FTPB + threadIdx.x;
    bool ok = false;
    if (c < total) {
      ok = true;
      if (RF != RF_NONE || ENV || DUR) {
        const int64_t row = cand_row(coff, start, nr, c);
        if (RF == RF_Z3) ok = z3_in_bounds(fdesc, (int16_t)bin[row], (int64_t)z[row]);
        if (RF == RF_Z2) {
          const int64_t zz = (int64_t)z[row];
          const int32_t x = z2_combine(zz), y = z2_combine(zz >> 1);
          bool in = false;
          for (int k = 0; k < nxy && !in; ++k) {
            const int32_t* q = fdesc + 4 * k;
            in = x >= q[0] && x <= q[2] && y >= q[1] && y <= q[3];
          }
          ok = in;
        }
        if ((ENV || DUR) && ok) {
          const int64_t r = ff.perm ? ff.perm[row] : row;
          if (DUR) {
            const int64_t t = ff.t[r];
            ok = t > ff.t_lo && t < ff.t_hi;
          }
          if (ENV && ok) {
            const double x0 = ff.xmin[r], y0 = ff.ymin[r], x1 = ff.xmax[r], y1 = ff.ymax[r];
            bool in = false;
            for (int k = 0; k < ff.nbox && !in; ++k) in = env_intersects(x0, y0, x1, y1, ff.boxes + 4 * k);
            ok = in;
          }
        }
      }
    }
    const uint64_t w = __ballot(ok);
    if (lane == 0) {
      const int64_t word = (base + (int64_t)u * FTPB + wave * 64) >> 6;
      if ((word << 6) < total) mask[word] = w;
      local += __popcll(w);
    }
  }
  block_count(local, block_counts);
}

// compacted candidate indices -> table rows (-> input rows through perm)
__global__ __launch_bounds__(FTPB) void k_cand_to_row(int64_t* __restrict__ ids, int64_t m,
                                                      const int64_t* __restrict__ coff, const int64_t* __restrict__ start,
                                                      int64_t nr, const int64_t* __restrict__ perm) {
  for (int64_t j = (int64_t)blockIdx.x * FTPB + threadIdx.x; j < m; j += (int64_t)gridDim.x * FTPB) {
    const int64_t row = cand_row(coff, start, nr, ids[j]);
    ids[j] = perm ? perm[row] : row;
  }
}

// ------------------------------------------------------------------ host side

static inline int32_t be32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3]);
}
static inline int16_t be16(const uint8_t* p) { return (int16_t)(uint16_t)((uint16_t)p[0] << 8 | p[1]); }

// bit spread with `stride` (2 or 3), the host mirror of Z2.split / Z3.split without masking
static uint64_t dilate(uint64_t v, int bits, int stride) {
  uint64_t o = 0;
  for (int i = 0; i < bits; ++i) o |= ((v >> i) & 1ull) << (stride * i);
  return o;
}

// Z3 boxes (xmin, ymin, xmax, ymax) as dilated (xlo, xhi, ylo, yhi); dims are 21-bit, non-negative
static void z3_dilated_boxes(const int32_t* xy, int nxy, std::vector<uint64_t>& out) {
  out.clear();
  const int64_t top = (1 << 21) - 1;
  for (int i = 0; i < nxy; ++i) {
    for (int d = 0; d < 2; ++d) {
      const int64_t lo = std::max<int64_t>(xy[4 * i + d], 0), hi = std::min<int64_t>(xy[4 * i + 2 + d], top);
      if (lo > hi || lo > top || hi < 0) { out.push_back(1ull << 63); out.push_back(0); continue; }   // empty
      out.push_back(dilate((uint64_t)lo, 21, 3) << d);
      out.push_back(dilate((uint64_t)hi, 21, 3) << d);
    }
  }
}

// Z2 boxes: signed 32-bit dims, top bit flipped into unsigned order
static void z2_dilated_boxes(const int32_t* xy, int nxy, std::vector<uint64_t>& out) {
  out.clear();
  for (int i = 0; i < nxy; ++i) {
    for (int d = 0; d < 2; ++d) {
      const int32_t lo = xy[4 * i + d], hi = xy[4 * i + 2 + d];
      if (lo > hi) { out.push_back(~0ull); out.push_back(0); continue; }   // empty
      out.push_back(dilate((uint32_t)lo ^ 0x80000000u, 32, 2) << d);
      out.push_back(dilate((uint32_t)hi ^ 0x80000000u, 32, 2) << d);
    }
  }
}

// Z3Filter.deserializeFromBytes (Z3Filter.scala:139-153) -> flat descriptor
static bool build_z3_desc(const uint8_t* b, size_t len, std::vector<int32_t>& d) {
  size_t o = 0;
  auto need = [&](size_t k) { return o + k <= len; };
  if (!need(4)) return false;
  const int32_t nxy = be32(b + o); o += 4;
  if (nxy < 0 || !need((size_t)nxy * 16)) return false;
  std::vector<int32_t> xy((size_t)nxy * 4);
  for (size_t i = 0; i < xy.size(); ++i) { xy[i] = be32(b + o); o += 4; }
  if (!need(4)) return false;
  const int32_t nt = be32(b + o); o += 4;
  if (nt < 0) return false;
  std::vector<int32_t> ep((size_t)nt * 2, 0), tiv;
  for (int k = 0; k < nt; ++k) {
    if (!need(4)) return false;
    const int32_t l = be32(b + o); o += 4;
    if (l == -1) { ep[2 * k] = -1; ep[2 * k + 1] = -1; continue; }   // null epoch: whole period
    if (l < 0 || !need((size_t)l * 8)) return false;
    ep[2 * k] = (int32_t)(tiv.size() / 2);
    for (int i = 0; i < 2 * l; ++i) { tiv.push_back(be32(b + o)); o += 4; }
    ep[2 * k + 1] = (int32_t)(tiv.size() / 2);
  }
  if (!need(4)) return false;
  const int16_t min_e = be16(b + o), max_e = be16(b + o + 2);
  d.clear();
  d.push_back(nxy);
  d.push_back(min_e);
  d.push_back(max_e);
  d.push_back(nt);
  d.push_back(0);
  d.insert(d.end(), xy.begin(), xy.end());
  d.insert(d.end(), ep.begin(), ep.end());
  d.insert(d.end(), tiv.begin(), tiv.end());
  return true;
}

}  // namespace gm

using namespace gm;

namespace gm {

// scratch buffers per call, carved from the context's scan workspace (stream-ordered reuse)
int alloc_scan(gm_ctx* ctx, int64_t n, uint64_t* user_mask, size_t desc_words, ScanBufs& b) {
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  const int64_t nwords = nblocks * (FROWS / 64);
  const size_t a_mask = user_mask ? 0 : (size_t)nwords * 8;
  const size_t a_cnt = ((size_t)nblocks * 4 + 4 + 15) & ~(size_t)15;
  const size_t a_off = ((size_t)(nblocks + 1) * 8 + 15) & ~(size_t)15;
  const size_t a_part = ((size_t)(nblocks / SCAN_CHUNK + 2) * 8 + 15) & ~(size_t)15;
  const size_t a_desc = (desc_words * 4 + 15) & ~(size_t)15;
  void* base = nullptr;
  int rc = ctx_workspace(ctx, WS_SCAN, a_mask + a_cnt + a_off + a_part + a_desc + 16, &base);
  if (rc) return rc;
  char* p = (char*)base;
  b.mask = user_mask ? user_mask : (uint64_t*)p;
  p += a_mask;
  b.counts = (int32_t*)p; p += a_cnt;
  b.offsets = (int64_t*)p; p += a_off;
  b.partials = (int64_t*)p; p += a_part;
  b.desc = desc_words ? (int32_t*)p : nullptr;
  return GM_OK;
}

void free_scan(gm_ctx*, uint64_t*, ScanBufs&) {}   // workspace memory stays with the context

// passes B and C + count readback
int finish_scan(gm_ctx* ctx, int64_t n, ScanBufs& b, int64_t* ids, int64_t ids_cap, int64_t* n_match) {
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  if (ids || n_match) {
    launch_excl_scan(ctx->stream, b.counts, nblocks, b.offsets, b.partials, b.offsets + nblocks);
    GM_CHECK_LAUNCH();
  }
  if (ids) {
    hipLaunchKernelGGL(k_mask_to_ids, dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, b.mask, n, b.offsets, ids,
                       ids_cap);
    GM_CHECK_LAUNCH();
  }
  if (n_match) {
    GM_HIP(hipMemcpyAsync(ctx->h_pinned, b.offsets + nblocks, 8, hipMemcpyDeviceToHost, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    *n_match = ctx->h_pinned[0];
  }
  return GM_OK;
}

}  // namespace gm

namespace {

// host mirror of the table's key order: (shard << 16 | bin as uint16, z as uint64)
struct HostRange {
  uint32_t kb_lo, kb_hi;
  uint64_t z_lo, z_hi;
};
inline bool h_lt(uint32_t ka, uint64_t za, uint32_t kb, uint64_t zb) { return ka < kb || (ka == kb && za < zb); }

}  // namespace

extern "C" {

int gm_z3filter_scan(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const int16_t* bin_ranges,
                     int n_bin_ranges, const int16_t* bin, const int64_t* z, int64_t n, uint64_t* mask,
                     int64_t* ids, int64_t ids_cap, int64_t* n_match) {
  if (!ctx || !filter_bytes || n < 0 || n_bin_ranges < 0) return GM_E_INVALID;
  std::vector<int32_t> desc;
  if (!build_z3_desc(filter_bytes, filter_len, desc)) {
    set_error("gm_z3filter_scan: malformed Z3Filter bytes");
    return GM_E_INVALID;
  }
  if (n == 0) { if (n_match) *n_match = 0; return GM_OK; }
  if (!bin || !z) return GM_E_INVALID;
  const int fwords = (int)desc.size();
  for (int i = 0; i < n_bin_ranges; ++i) { desc.push_back(bin_ranges[2 * i]); desc.push_back(bin_ranges[2 * i + 1]); }
  // device layout: [dilated boxes u64 x 4 nxy][descriptor][bin ranges]
  std::vector<uint64_t> dil;
  z3_dilated_boxes(desc.data() + 5, desc[0], dil);
  std::vector<int32_t> buf(2 * dil.size() + desc.size());
  if (!dil.empty()) memcpy(buf.data(), dil.data(), dil.size() * 8);
  memcpy(buf.data() + 2 * dil.size(), desc.data(), desc.size() * 4);
  ScanBufs b;
  int rc = alloc_scan(ctx, n, mask, buf.size(), b);
  if (rc) return rc;
  GM_HIP(hipMemcpyAsync(b.desc, buf.data(), buf.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));  // buf is pageable host memory
  const uint64_t* d_dil = (const uint64_t*)b.desc;
  const int32_t* d_desc = b.desc + 2 * dil.size();
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  const size_t lds = desc.size() * 4;
  const bool fast = desc[0] <= FBOX && n_bin_ranges <= FBIN;
  if (aligned16(bin) && aligned16(z) && fast)
    hipLaunchKernelGGL(k_z3filter_mask_v<true>, dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, (const sv2*)bin,
                       (const lv2*)z, n, d_dil, d_desc, d_desc + fwords, n_bin_ranges, b.mask, b.counts);
  else if (aligned16(bin) && aligned16(z))
    hipLaunchKernelGGL(k_z3filter_mask_v<false>, dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, (const sv2*)bin,
                       (const lv2*)z, n, d_dil, d_desc, d_desc + fwords, n_bin_ranges, b.mask, b.counts);
  else
    hipLaunchKernelGGL(k_z3filter_mask, dim3((unsigned)nblocks), dim3(FTPB), lds, ctx->stream, bin, z, n, d_desc,
                       fwords, d_desc + fwords, n_bin_ranges, b.mask, b.counts);
  GM_CHECK_LAUNCH();
  rc = finish_scan(ctx, n, b, ids, ids_cap, n_match);
  free_scan(ctx, mask, b);
  if (rc) return rc;
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

int gm_z2filter_scan(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const int64_t* z, int64_t n,
                     uint64_t* mask, int64_t* ids, int64_t ids_cap, int64_t* n_match) {
  if (!ctx || !filter_bytes || n < 0 || filter_len < 4) return GM_E_INVALID;
  const int32_t nxy = be32(filter_bytes);
  if (nxy < 0 || 4 + (size_t)nxy * 16 > filter_len) {
    set_error("gm_z2filter_scan: malformed Z2Filter bytes");
    return GM_E_INVALID;
  }
  if (n == 0) { if (n_match) *n_match = 0; return GM_OK; }
  if (!z) return GM_E_INVALID;
  std::vector<int32_t> xy((size_t)nxy * 4);
  for (size_t i = 0; i < xy.size(); ++i) xy[i] = be32(filter_bytes + 4 + 4 * i);
  // device layout: [dilated boxes u64 x 4 nxy][boxes int32 x 4 nxy]
  std::vector<uint64_t> dil;
  z2_dilated_boxes(xy.data(), nxy, dil);
  std::vector<int32_t> buf(2 * dil.size() + xy.size() + 1);
  if (!dil.empty()) memcpy(buf.data(), dil.data(), dil.size() * 8);
  if (!xy.empty()) memcpy(buf.data() + 2 * dil.size(), xy.data(), xy.size() * 4);
  ScanBufs b;
  int rc = alloc_scan(ctx, n, mask, buf.size(), b);
  if (rc) return rc;
  GM_HIP(hipMemcpyAsync(b.desc, buf.data(), buf.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  const uint64_t* d_dil = (const uint64_t*)b.desc;
  const int32_t* d_xy = b.desc + 2 * dil.size();
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  if (aligned16(z) && nxy <= FBOX)
    hipLaunchKernelGGL(k_z2filter_mask_v<true>, dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, (const lv2*)z, n,
                       d_dil, d_xy, nxy, b.mask, b.counts);
  else if (aligned16(z))
    hipLaunchKernelGGL(k_z2filter_mask_v<false>, dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, (const lv2*)z, n,
                       d_dil, d_xy, nxy, b.mask, b.counts);
  else
    hipLaunchKernelGGL(k_z2filter_mask, dim3((unsigned)nblocks), dim3(FTPB), xy.size() * 4 + 4, ctx->stream, z, n,
                       d_xy, nxy, b.mask, b.counts);
  GM_CHECK_LAUNCH();
  rc = finish_scan(ctx, n, b, ids, ids_cap, n_match);
  free_scan(ctx, mask, b);
  if (rc) return rc;
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

// shared driver of gm_z3filter_scan_rows / gm_z2filter_scan_rows
static int filter_rows(gm_ctx* ctx, bool z3, const std::vector<int32_t>& desc, const uint8_t* rows,
                       const int64_t* row_off, int key_offset, int64_t n, uint64_t* mask, int64_t* ids,
                       int64_t ids_cap, int64_t* n_match, int64_t* n_short) {
  if (n == 0) { if (n_match) *n_match = 0; if (n_short) *n_short = 0; return GM_OK; }
  if (!rows || !row_off || key_offset < 0) return GM_E_INVALID;
  ScanBufs b;
  // descriptor words, then one 8-B short-row counter (16-B aligned)
  const size_t dw = (desc.size() + 3) & ~(size_t)3;
  int rc = alloc_scan(ctx, n, mask, dw + 4, b);
  if (rc) return rc;
  unsigned long long* d_short = (unsigned long long*)(b.desc + dw);
  GM_HIP(hipMemcpyAsync(b.desc, desc.data(), desc.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipMemsetAsync(d_short, 0, 8, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));  // desc is pageable host memory
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  const size_t lds = std::max<size_t>(desc.size() * 4, 4);
  if (z3)
    hipLaunchKernelGGL(k_filter_rows_mask<true>, dim3((unsigned)nblocks), dim3(FTPB), lds, ctx->stream, rows, row_off,
                       key_offset, n, b.desc, (int)desc.size(), b.mask, b.counts, d_short);
  else
    hipLaunchKernelGGL(k_filter_rows_mask<false>, dim3((unsigned)nblocks), dim3(FTPB), lds, ctx->stream, rows, row_off,
                       key_offset, n, b.desc, (int)desc.size(), b.mask, b.counts, d_short);
  GM_CHECK_LAUNCH();
  rc = finish_scan(ctx, n, b, ids, ids_cap, n_match);
  if (rc) return rc;
  if (n_short) {
    GM_HIP(hipMemcpyAsync(ctx->h_pinned, d_short, 8, hipMemcpyDeviceToHost, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    *n_short = ctx->h_pinned[0];
  }
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

int gm_z3filter_scan_rows(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const uint8_t* rows,
                          const int64_t* row_off, int key_offset, int64_t n, uint64_t* mask, int64_t* ids,
                          int64_t ids_cap, int64_t* n_match, int64_t* n_short) {
  if (!ctx || !filter_bytes || n < 0) return GM_E_INVALID;
  std::vector<int32_t> desc;
  if (!build_z3_desc(filter_bytes, filter_len, desc)) {
    set_error("gm_z3filter_scan_rows: malformed Z3Filter bytes");
    return GM_E_INVALID;
  }
  return filter_rows(ctx, true, desc, rows, row_off, key_offset, n, mask, ids, ids_cap, n_match, n_short);
}

int gm_z2filter_scan_rows(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const uint8_t* rows,
                          const int64_t* row_off, int key_offset, int64_t n, uint64_t* mask, int64_t* ids,
                          int64_t ids_cap, int64_t* n_match, int64_t* n_short) {
  if (!ctx || !filter_bytes || n < 0 || filter_len < 4) return GM_E_INVALID;
  const int32_t nxy = be32(filter_bytes);
  if (nxy < 0 || 4 + (size_t)nxy * 16 > filter_len) {
    set_error("gm_z2filter_scan_rows: malformed Z2Filter bytes");
    return GM_E_INVALID;
  }
  std::vector<int32_t> xy((size_t)nxy * 4);
  for (size_t i = 0; i < xy.size(); ++i) xy[i] = be32(filter_bytes + 4 + 4 * i);
  return filter_rows(ctx, false, xy, rows, row_off, key_offset, n, mask, ids, ids_cap, n_match, n_short);
}

int gm_strict_scan(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n, const double* bbox,
                   int has_during, int64_t lo, int64_t hi, uint64_t* mask, int64_t* ids, int64_t ids_cap,
                   int64_t* n_match) {
  if (!ctx || !bbox || n < 0) return GM_E_INVALID;
  if (n == 0) { if (n_match) *n_match = 0; return GM_OK; }
  if (!x || !y || (has_during && !t_ms)) return GM_E_INVALID;
  ScanBufs b;
  int rc = alloc_scan(ctx, n, mask, 0, b);
  if (rc) return rc;
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  if (aligned16(x) && aligned16(y) && (!has_during || aligned16(t_ms))) {
    const dv2* x2 = (const dv2*)x;
    const dv2* y2 = (const dv2*)y;
    const lv2* t2 = (const lv2*)t_ms;
    uint64_t* m8 = b.mask;
    if (has_during)
      hipLaunchKernelGGL((k_strict_mask_v<true>), dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, x2, y2, t2, n,
                         bbox[0], bbox[1], bbox[2], bbox[3], lo, hi, m8, b.counts);
    else
      hipLaunchKernelGGL((k_strict_mask_v<false>), dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, x2, y2, t2, n,
                         bbox[0], bbox[1], bbox[2], bbox[3], lo, hi, m8, b.counts);
  } else if (has_during)
    hipLaunchKernelGGL((k_strict_mask<true>), dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, x, y, t_ms, n,
                       bbox[0], bbox[1], bbox[2], bbox[3], lo, hi, b.mask, b.counts);
  else
    hipLaunchKernelGGL((k_strict_mask<false>), dim3((unsigned)nblocks), dim3(FTPB), 0, ctx->stream, x, y, t_ms, n,
                       bbox[0], bbox[1], bbox[2], bbox[3], lo, hi, b.mask, b.counts);
  GM_CHECK_LAUNCH();
  rc = finish_scan(ctx, n, b, ids, ids_cap, n_match);
  free_scan(ctx, mask, b);
  if (rc) return rc;
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

int gm_table_scan(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                  const gm_key_range* ranges, int64_t n_ranges, const gm_scan_filter* f, const int64_t* perm,
                  int64_t* ids, int64_t ids_cap, int64_t* n_match, int64_t* n_scanned) {
  if (!ctx || n < 0 || n_ranges < 0 || (n_ranges > 0 && !ranges) || ids_cap < 0) return GM_E_INVALID;
  if (n > 0 && !z) return GM_E_INVALID;
  gm_scan_filter none{};
  if (!f) f = &none;
  if (f->z3filter && f->z2filter) return set_error("gm_table_scan: a Z3Filter and a Z2Filter together"), GM_E_INVALID;
  if (f->z3filter && !bin) return set_error("gm_table_scan: a Z3Filter needs the bin column"), GM_E_INVALID;
  const bool env = f->n_boxes > 0, dur = f->during != 0;
  if (f->n_boxes < 0 || (env && (!f->boxes || !f->xmin || !f->ymin || !f->xmax || !f->ymax)) || (dur && !f->t_ms))
    return GM_E_INVALID;
  // the row filter's descriptor: Z3Filter.deserializeFromBytes or Z2Filter's boxes
  std::vector<int32_t> desc;
  int rf = RF_NONE, nxy = 0;
  if (f->z3filter) {
    if (!build_z3_desc(f->z3filter, f->z3filter_len, desc)) {
      set_error("gm_table_scan: malformed Z3Filter bytes");
      return GM_E_INVALID;
    }
    rf = RF_Z3;
  } else if (f->z2filter) {
    if (f->z2filter_len < 4) return GM_E_INVALID;
    nxy = be32(f->z2filter);
    if (nxy < 0 || 4 + (size_t)nxy * 16 > f->z2filter_len) {
      set_error("gm_table_scan: malformed Z2Filter bytes");
      return GM_E_INVALID;
    }
    for (int i = 0; i < 4 * nxy; ++i) desc.push_back(be32(f->z2filter + 4 + 4 * i));
    rf = RF_Z2;
  }
  // the BatchScanner's view of the ranges: sorted, overlapping / adjacent ones merged
  std::vector<HostRange> rs;
  rs.reserve((size_t)n_ranges);
  for (int64_t i = 0; i < n_ranges; ++i) {
    const gm_key_range& r = ranges[i];
    HostRange h{((uint32_t)r.shard << 16) | (uint16_t)r.bin_lo, ((uint32_t)r.shard << 16) | (uint16_t)r.bin_hi,
                (uint64_t)r.z_lo, (uint64_t)r.z_hi};
    if (h_lt(h.kb_hi, h.z_hi, h.kb_lo, h.z_lo)) continue;  // empty
    rs.push_back(h);
  }
  std::sort(rs.begin(), rs.end(), [](const HostRange& a, const HostRange& b) { return h_lt(a.kb_lo, a.z_lo, b.kb_lo, b.z_lo); });
  std::vector<DevRange> dr;
  for (const HostRange& h : rs) {
    if (!dr.empty()) {
      DevRange& last = dr.back();
      // merge when h.lo <= last.hi + 1 in key order
      const bool le = !h_lt(last.kb_hi, last.z_hi, h.kb_lo, h.z_lo) ||
                      (last.z_hi != ~0ull && last.kb_hi == h.kb_lo && last.z_hi + 1 == h.z_lo) ||
                      (last.z_hi == ~0ull && h.z_lo == 0 && last.kb_hi + 1 == h.kb_lo);
      if (le) {
        if (h_lt(last.kb_hi, last.z_hi, h.kb_hi, h.z_hi)) { last.kb_hi = h.kb_hi; last.z_hi = h.z_hi; }
        continue;
      }
    }
    dr.push_back(DevRange{h.z_lo, h.z_hi, h.kb_lo, h.kb_hi});
  }
  const int64_t nr = (int64_t)dr.size();
  if (n == 0 || nr == 0) {
    if (n_match) *n_match = 0;
    if (n_scanned) *n_scanned = 0;
    return GM_OK;
  }
  hipStream_t s = ctx->stream;
  DevRange* d_rg = nullptr;
  int64_t *start = nullptr, *coff = nullptr;
  GM_HIP(hipMallocAsync((void**)&d_rg, (size_t)nr * sizeof(DevRange), s));
  GM_HIP(hipMallocAsync((void**)&start, (size_t)nr * 8, s));
  GM_HIP(hipMallocAsync((void**)&coff, (size_t)(nr + 1) * 8, s));
  int crc = copy_h2d(ctx, d_rg, dr.data(), (size_t)nr * sizeof(DevRange));
  if (crc) return crc;
  hipLaunchKernelGGL(k_range_bounds, dim3((unsigned)((nr + FTPB - 1) / FTPB)), dim3(FTPB), 0, s, shard,
                     (const uint16_t*)bin, (const uint64_t*)z, n, d_rg, nr, start, coff);
  hipLaunchKernelGGL(k_scan_i64, dim3(1), dim3(1024), 0, s, coff, nr);
  GM_CHECK_LAUNCH();
  GM_HIP(hipMemcpyAsync(ctx->h_pinned, coff + nr, 8, hipMemcpyDeviceToHost, s));
  GM_HIP(hipStreamSynchronize(s));  // dr is pageable; the candidate count sizes the pass below
  const int64_t total = ctx->h_pinned[0];
  if (n_scanned) *n_scanned = total;
  int rc = GM_OK;
  int64_t nm = 0;
  if (total > 0) {
    // device descriptor: [query boxes f64 x 4 nbox][row-filter words]
    const size_t box_words = env ? (size_t)f->n_boxes * 8 : 0;
    std::vector<int32_t> buf(box_words + desc.size());
    if (env) memcpy(buf.data(), f->boxes, (size_t)f->n_boxes * 32);
    if (!desc.empty()) memcpy(buf.data() + box_words, desc.data(), desc.size() * 4);
    ScanBufs b;
    rc = alloc_scan(ctx, total, nullptr, buf.size() + 4, b);
    if (!rc) {
      if (!buf.empty()) {
        GM_HIP(hipMemcpyAsync(b.desc, buf.data(), buf.size() * 4, hipMemcpyHostToDevice, s));
        GM_HIP(hipStreamSynchronize(s));
      }
      FullFilter ff{f->xmin, f->ymin, f->xmax, f->ymax, f->t_ms, env ? (const double*)b.desc : nullptr, f->n_boxes,
                    f->t_lo, f->t_hi, perm};
      const int32_t* d_desc = b.desc + box_words;
      const int64_t nblocks = (total + FROWS - 1) / FROWS;
      void (*kern)(const uint16_t*, const uint64_t*, const int64_t*, const int64_t*, int64_t, int64_t, const int32_t*,
                   int, FullFilter, uint64_t*, int32_t*) = nullptr;
#define GM_RANGE_MASK(R)                                                                   \
  (env ? (dur ? k_range_mask<R, true, true> : k_range_mask<R, true, false>)               \
       : (dur ? k_range_mask<R, false, true> : k_range_mask<R, false, false>))
      kern = rf == RF_Z3 ? GM_RANGE_MASK(RF_Z3) : rf == RF_Z2 ? GM_RANGE_MASK(RF_Z2) : GM_RANGE_MASK(RF_NONE);
#undef GM_RANGE_MASK
      hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(FTPB), 0, s, (const uint16_t*)bin, (const uint64_t*)z, coff,
                         start, nr, total, d_desc, nxy, ff, b.mask, b.counts);
      if (hipGetLastError() != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "k_range_mask");
      if (!rc) rc = finish_scan(ctx, total, b, ids, ids_cap, &nm);
      if (!rc && ids && nm > 0) {
        const int64_t m = std::min(nm, ids_cap);
        hipLaunchKernelGGL(k_cand_to_row, dim3((unsigned)std::min<int64_t>(4096, (m + FTPB - 1) / FTPB)), dim3(FTPB), 0,
                           s, ids, m, coff, start, nr, perm);
        if (hipGetLastError() != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "k_cand_to_row");
      }
      free_scan(ctx, nullptr, b);
    }
  }
  (void)hipFreeAsync(d_rg, s);
  (void)hipFreeAsync(start, s);
  (void)hipFreeAsync(coff, s);
  if (rc) return rc;
  if (n_match) *n_match = nm;
  if (ids && nm > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

int gm_key_range_scan(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                      const gm_key_range* ranges, int64_t n_ranges, const uint8_t* filter_bytes, size_t filter_len,
                      const int64_t* perm, int64_t* ids, int64_t ids_cap, int64_t* n_match, int64_t* n_scanned) {
  if (!ctx) return GM_E_INVALID;
  if (n > 0 && !bin) return GM_E_INVALID;
  gm_scan_filter f{};
  f.z3filter = filter_bytes;
  f.z3filter_len = filter_len;
  return gm_table_scan(ctx, shard, bin, z, n, ranges, n_ranges, &f, perm, ids, ids_cap, n_match, n_scanned);
}

}  // extern "C"
