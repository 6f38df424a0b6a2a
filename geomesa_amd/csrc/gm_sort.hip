// gm_sort.hip -- the sorted key table: row-key bytes, device sort into table order, and range scans.
//
// A GeoMesa Z3 table is the set of row keys [shard?][bin BE16][z BE64][id] kept in byte order by the
// store (Z3IndexKeySpace.toIndexKey, idx/index/z3/Z3IndexKeySpace.scala:63-95; ByteArrays.writeShort /
// writeLong, geomesa-utils/.../index/ByteArrays.scala:51,90-99).  A query seeks each byte range
// getRangeBytes produces (Z3IndexKeySpace.scala:196-238) and the tablet server runs the Z3Filter on
// every row inside (RowFilterIterator.scala:52-66).  Here the table is columnar and resident in HBM:
//   * gm_z3_key_bytes  -- the row-key prefix bytes, staged through LDS so the stores are 16-B wide;
//   * gm_sort_keys     -- a stable sort of (shard u8, bin u16, z u64) in that byte order.  The key
//                         K = shard:bin:z is an 88-bit integer; one read finds its varying bits (OR /
//                         AND).  Three stable digit passes (8-bit digits, per-block segments:
//                         histogram -> one-block scan -> scatter, wave ballots rank equal digits, LDS
//                         reorders each 8192-row tile so the global writes are digit runs) order the
//                         rows by the top 24 varying bits; then k_sort_local ranks every run of
//                         equal 24-bit prefixes (~15 rows for 250M uniform keys) by full key in LDS
//                         and writes the rows to their final places.  A run longer than 1024 rows
//                         (skewed keys) sends the call to digit passes over every varying byte (LSD,
//                         the same kernels), which is also GM_PARAM_SORT_MODE 1;
// The range scan over a sorted table (gm_key_range_scan) lives with the other row-filter scans in
// gm_filter.hip.
#include <string.h>

#include <algorithm>
#include <vector>

#include "gm_scan.hpp"

namespace gm {

constexpr int STPB = 256;               // sort / scan threads per block
constexpr int NPASS = 11;               // digit positions: z bytes 0..7, bin bytes 0..1, shard

// 24 bits of K = bs:z (bs = bin | shard << 16) from bit `off` (0 <= off < 88) up; a digit is the low 8
__device__ __forceinline__ uint32_t key_bits(uint32_t bs, uint64_t z, int off) {
  uint64_t v;
  if (off >= 64) v = (uint64_t)bs >> (off - 64);
  else {
    v = z >> off;
    if (off > 0) v |= (uint64_t)bs << (64 - off);
  }
  return (uint32_t)v & 0xffffffu;
}
__device__ __forceinline__ uint32_t key_digit(uint32_t bs, uint64_t z, int off) { return key_bits(bs, z, off) & 255u; }

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// which digit passes carry information: the OR and the AND of every key column (a digit on which
// OR == AND is the same for every key, so its pass would be the identity and is skipped).
// acc[0] = OR z, acc[1] = OR (bin | shard << 16), acc[2] = AND z, acc[3] = AND (bin | shard << 16).
__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_and(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v &= __shfl_xor(v, o, 64);
  return v;
}
__global__ __launch_bounds__(STPB) void k_key_or_and(const uint8_t* __restrict__ sh, const uint16_t* __restrict__ bin,
                                                     const uint64_t* __restrict__ z, int64_t n,
                                                     unsigned long long* __restrict__ acc, int vec) {
  uint64_t zo = 0, za = ~0ull, bo = 0, ba = ~0ull;
  const int64_t np = n >> 1;   // pairs: 16-B z loads
  for (int64_t p = (int64_t)blockIdx.x * STPB + threadIdx.x; p < np; p += (int64_t)gridDim.x * STPB) {
    uint64_t z0, z1, b0, b1;
    if (vec) {
      const ulonglong2 zz = *(const ulonglong2*)(z + 2 * p);
      const ushort2 bb = *(const ushort2*)(bin + 2 * p);
      z0 = zz.x; z1 = zz.y; b0 = bb.x; b1 = bb.y;
      if (sh) { const uchar2 ss = *(const uchar2*)(sh + 2 * p); b0 |= (uint64_t)ss.x << 16; b1 |= (uint64_t)ss.y << 16; }
    } else {
      z0 = z[2 * p]; z1 = z[2 * p + 1]; b0 = bin[2 * p]; b1 = bin[2 * p + 1];
      if (sh) { b0 |= (uint64_t)sh[2 * p] << 16; b1 |= (uint64_t)sh[2 * p + 1] << 16; }
    }
    zo |= z0 | z1; za &= z0 & z1;
    bo |= b0 | b1; ba &= b0 & b1;
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t b0 = (uint64_t)bin[n - 1] | (sh ? (uint64_t)sh[n - 1] << 16 : 0);
    zo |= z[n - 1]; za &= z[n - 1]; bo |= b0; ba &= b0;
  }
  zo = wave_or(zo); za = wave_and(za); bo = wave_or(bo); ba = wave_and(ba);
  if ((threadIdx.x & 63) == 0) {
    atomicOr(&acc[0], zo); atomicOr(&acc[1], bo); atomicAnd(&acc[2], za); atomicAnd(&acc[3], ba);
  }
}

// per-block segment histogram of one digit (bits [off, off + 8) of K), digit-major:
// hist[d * gridDim.x + block].  1024 threads, two rows per lane (16-B z loads), only the columns the
// digit touches are read, per-wave LDS counters summed at the end.
constexpr int HT = 1024;
__global__ __launch_bounds__(HT) void k_sort_hist(const uint8_t* __restrict__ sh, const uint16_t* __restrict__ bin,
                                                  const uint64_t* __restrict__ z, int64_t n, int64_t per_block,
                                                  int off, uint32_t* __restrict__ hist, int vec) {
  __shared__ uint32_t h[HT / 64][256];
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (HT / 64) * 256; i += HT) (&h[0][0])[i] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(n, b0 + per_block);
  const bool nz = off < 64, nb = off + 8 > 64 && off < 80, ns = sh != nullptr && off + 8 > 80;
  // full stretches: 4 pairs per lane, loads issued together (a digit extraction between loads made
  // the compiler wait for each pair before the next load)
  constexpr int HU = 4;
  int64_t i = b0 + 2 * threadIdx.x;
  if (vec)
    for (; i + 2 * HT * (HU - 1) + 1 < b1; i += 2 * HT * HU) {
      ulonglong2 zz[HU];
      uint32_t bb[HU], ss[HU];
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        zz[u] = nz ? *(const ulonglong2*)(z + i + 2 * HT * u) : make_ulonglong2(0ull, 0ull);
        bb[u] = nb ? *(const uint32_t*)(bin + i + 2 * HT * u) : 0u;
        ss[u] = ns ? (uint32_t)*(const uint16_t*)(sh + i + 2 * HT * u) : 0u;
      }
#pragma unroll
      for (int u = 0; u < HU; ++u) {
        atomicAdd(&h[wave][key_digit((bb[u] & 0xffffu) | ((ss[u] & 0xffu) << 16), zz[u].x, off)], 1u);
        atomicAdd(&h[wave][key_digit((bb[u] >> 16) | ((ss[u] >> 8) << 16), zz[u].y, off)], 1u);
      }
    }
  for (; i < b1; i += 2 * HT) {   // b0 is even (tile multiple)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t r = i + e;
      if (r >= b1) continue;
      const uint32_t bs = (nb ? (uint32_t)bin[r] : 0u) | (ns ? (uint32_t)sh[r] << 16 : 0u);
      atomicAdd(&h[wave][key_digit(bs, nz ? z[r] : 0ull, off)], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < HT / 64; ++w) c += h[w][threadIdx.x];
    hist[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = c;
  }
}

// Stable scatter of one digit pass, one 1024-thread workgroup per CU.  Each block walks its segment
// in 8192-row tiles; wave w owns rows [512 w, 512 w + 512) of a tile and reads them in 4 slots of
// 128 rows, 2 per lane (16-B z loads).  Within a slot, lanes holding the same digit find each other
// with 16 ballots (8 digit bits x even / odd row); a per-wave LDS counter per digit turns slot ranks
// into wave ranks, a scan over the waves into block ranks, so a row's place in the tile is (digit,
// wave, slot, lane, even/odd) = stable.  The tile is reordered in LDS and leaves as digit runs at
// the block's cursor for each digit (runs average 32 rows for uniform digits: 256-B z segments).
#ifndef GM_SORT_BT
#define GM_SORT_BT 1024
#endif
constexpr int BT = GM_SORT_BT;      // scatter threads per block
constexpr int BW = BT / 64;         // waves
constexpr int BSLOT = 4;            // slots of 2 rows per lane
constexpr int BTILE = BT * 2 * BSLOT;   // 8192 rows per tile

__device__ __forceinline__ uint64_t digit_mask(const uint64_t* bal, uint32_t d) {
  uint64_t m = ~0ull;
#pragma unroll
  for (int bit = 0; bit < 8; ++bit) m &= ((d >> bit) & 1u) ? bal[bit] : ~bal[bit];
  return m;
}

// SH: a shard column; PIN: a permutation input (else the row index).  The next tile's loads only issue
// into raw registers (z pair, bin pair, shard pair, permutation pair) and are combined when ranked:
// a combine (or a column test) between loads made the compiler wait for each slot's loads before
// issuing the next ones, which serialised the "prefetch" into four round trips per tile.
template <bool SH, bool PIN>
__global__ __launch_bounds__(BT) void k_sort_scatter(const uint8_t* __restrict__ sh_in, const uint16_t* __restrict__ bin_in,
                                                     const uint64_t* __restrict__ z_in,
                                                     const uint32_t* __restrict__ perm_in, uint8_t* __restrict__ sh_out,
                                                     uint16_t* __restrict__ bin_out, uint64_t* __restrict__ z_out,
                                                     uint32_t* __restrict__ perm_out, int64_t* __restrict__ perm64_out,
                                                     int64_t n, int64_t per_block, int doff,
                                                     const uint32_t* __restrict__ off, int vec) {
  __shared__ uint64_t s_z[BTILE];
  __shared__ uint32_t s_perm[BTILE];
  __shared__ uint16_t s_bin[BTILE];
  __shared__ uint8_t s_sh[SH ? BTILE : 1];
  __shared__ uint16_t s_wcnt[BW][256];      // per wave: rows of each digit so far (then: wave offsets)
  __shared__ uint32_t s_gcur[256], s_tot[256], s_dstart[256], s_wsum[4];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t < 256) s_gcur[t] = off[(int64_t)t * gridDim.x + blockIdx.x];
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(n, b0 + per_block);
  const uint64_t lt = lanemask_lt();
  // raw loads of this lane's rows of a tile (2 rows per slot)
  ulonglong2 rz[BSLOT];
  uint32_t rb[BSLOT];    // bin pair (ushort2 bits)
  uint32_t rs[BSLOT];    // shard pair (uchar2 bits)
  uint2 rp[BSLOT];       // permutation pair
  auto load = [&](int64_t t0) __attribute__((always_inline)) {
    const bool full = vec && t0 + BTILE <= b1;   // block-uniform: every slot holds two rows
    if (full) {
#pragma unroll
      for (int k = 0; k < BSLOT; ++k) {
        const int64_t i = t0 + wave * (2 * 64 * BSLOT) + k * 128 + 2 * lane;
        rz[k] = *(const ulonglong2*)(z_in + i);
        rb[k] = *(const uint32_t*)(bin_in + i);
        if (SH) rs[k] = *(const uint16_t*)(sh_in + i);
        if (PIN) rp[k] = *(const uint2*)(perm_in + i);
      }
    } else {
#pragma unroll
      for (int k = 0; k < BSLOT; ++k) {
        const int64_t i = t0 + wave * (2 * 64 * BSLOT) + k * 128 + 2 * lane;
        const bool ok0 = i < b1, ok1 = i + 1 < b1;
        rz[k].x = ok0 ? z_in[i] : 0; rz[k].y = ok1 ? z_in[i + 1] : 0;
        rb[k] = (ok0 ? (uint32_t)bin_in[i] : 0u) | ((ok1 ? (uint32_t)bin_in[i + 1] : 0u) << 16);
        if (SH) rs[k] = (ok0 ? (uint32_t)sh_in[i] : 0u) | ((ok1 ? (uint32_t)sh_in[i + 1] : 0u) << 8);
        if (PIN) rp[k] = make_uint2(ok0 ? perm_in[i] : 0u, ok1 ? perm_in[i + 1] : 0u);
      }
    }
  };
  if (b0 < b1) load(b0);
  for (int64_t t0 = b0; t0 < b1; t0 += BTILE) {
    // this tile's rows out of the raw registers
    uint64_t zv[BSLOT][2];
    uint32_t pv[BSLOT][2];
    uint32_t bs[BSLOT][2];   // bin | shard << 16
#pragma unroll
    for (int k = 0; k < BSLOT; ++k) {
      const int64_t i = t0 + wave * (2 * 64 * BSLOT) + k * 128 + 2 * lane;
      zv[k][0] = rz[k].x; zv[k][1] = rz[k].y;
      bs[k][0] = (rb[k] & 0xffffu) | (SH ? (rs[k] & 0xffu) << 16 : 0u);
      bs[k][1] = (rb[k] >> 16) | (SH ? ((rs[k] >> 8) & 0xffu) << 16 : 0u);
      if (PIN) { pv[k][0] = rp[k].x; pv[k][1] = rp[k].y; }
      else { pv[k][0] = (uint32_t)i; pv[k][1] = (uint32_t)(i + 1); }
    }
    for (int i = t; i < BW * 256 / 2; i += BT) ((uint32_t*)&s_wcnt[0][0])[i] = 0u;
    __syncthreads();
    uint32_t rd[BSLOT][2];   // wave rank | digit << 16; rank 0xffff = no row
#pragma unroll
    for (int k = 0; k < BSLOT; ++k) {
      const int64_t i = t0 + wave * (2 * 64 * BSLOT) + k * 128 + 2 * lane;
      const bool ok0 = i < b1, ok1 = i + 1 < b1;
      const uint32_t d0 = key_digit(bs[k][0], zv[k][0], doff);
      const uint32_t d1 = key_digit(bs[k][1], zv[k][1], doff);
      uint64_t bal0[8], bal1[8];
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        bal0[bit] = __ballot((d0 >> bit) & 1u);
        bal1[bit] = __ballot((d1 >> bit) & 1u);
      }
      const uint64_t okm0 = __ballot(ok0), okm1 = __ballot(ok1);
      // masks of lanes whose even / odd row holds my even / odd row's digit
      const uint64_t m00 = digit_mask(bal0, d0) & okm0, m01 = digit_mask(bal1, d0) & okm1;
      const uint64_t m10 = digit_mask(bal0, d1) & okm0, m11 = digit_mask(bal1, d1) & okm1;
      const uint64_t le = lt | (1ull << lane);
      const int r0 = __popcll(m00 & lt) + __popcll(m01 & lt);
      const int r1 = __popcll(m10 & le) + __popcll(m11 & lt);
      // wave counters: read before this slot's increments, then the first row of each digit adds
      const uint32_t c0 = s_wcnt[wave][d0], c1 = s_wcnt[wave][d1];
      rd[k][0] = (ok0 ? c0 + r0 : 0xffffu) | (d0 << 16);
      rd[k][1] = (ok1 ? c1 + r1 : 0xffffu) | (d1 << 16);
      __builtin_amdgcn_wave_barrier();
      if (ok0 && r0 == 0) s_wcnt[wave][d0] = (uint16_t)(c0 + __popcll(m00) + __popcll(m01));
      if (ok1 && r1 == 0) s_wcnt[wave][d1] = (uint16_t)(c1 + __popcll(m10) + __popcll(m11));
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    uint32_t run = 0, x = 0;
    if (t < 256) {   // per digit: exclusive offsets over the waves, and the digit's tile total
#pragma unroll
      for (int w = 0; w < BW; ++w) {
        const uint32_t c = s_wcnt[w][t];
        s_wcnt[w][t] = (uint16_t)run;
        run += c;
      }
      s_tot[t] = run;
      x = run;   // inclusive scan of the digit totals within the wave (waves 0-3 hold the 256 digits)
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) s_wsum[wave] = x;
    }
    __syncthreads();
    if (t < 256) {
      uint32_t pre = 0;
      for (int w = 0; w < wave; ++w) pre += s_wsum[w];
      s_dstart[t] = pre + x - run;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BSLOT; ++k) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint32_t r = rd[k][e] & 0xffffu, d = rd[k][e] >> 16;
        if (r == 0xffffu) continue;
        const uint32_t pos = s_dstart[d] + s_wcnt[wave][d] + r;
        s_z[pos] = zv[k][e]; s_bin[pos] = (uint16_t)bs[k][e];
        if (SH) s_sh[pos] = (uint8_t)(bs[k][e] >> 16);
        s_perm[pos] = pv[k][e];
      }
    }
    __syncthreads();
    if (t0 + BTILE < b1) load(t0 + BTILE);   // issued before the write-out: in flight during it
    const int cnt = (int)min((int64_t)BTILE, b1 - t0);
    for (int q = t; q < cnt; q += BT) {
      const uint32_t d = key_digit((uint32_t)s_bin[q] | (SH ? (uint32_t)s_sh[q] << 16 : 0u), s_z[q], doff);
      const int64_t g = (int64_t)s_gcur[d] + (q - (int)s_dstart[d]);
      z_out[g] = s_z[q];
      bin_out[g] = s_bin[q];
      if (SH) sh_out[g] = s_sh[q];
      if (perm64_out) perm64_out[g] = s_perm[q];
      else perm_out[g] = s_perm[q];
    }
    __syncthreads();
    if (t < 256) s_gcur[t] += s_tot[t];
  }
}

// Final placement after the prefix passes: the digit passes at bit offsets o1 > o2 > ... (each digit
// ends at a varying bit, and only constant bits lie between them) leave the rows grouped, stably, by
// P = digit(o1) : digit(o2) : ... -- the key's top varying bits, ~log2(n) + 3 of them, so that runs
// of equal P are short (Poisson(n / 2^bits) for uniform keys).  Tile k covers the runs of
// equal P that start in [k LSTEP, (k + 1) LSTEP); its rows are staged in LDS, a block scan marks each
// row's run (start, and at the start its end), each row counts the rows of its run with a smaller key
// (ties by position: stable) and goes to run start + rank: O(run length) LDS reads per row.  A run
// longer than RUN_MAX rows (skewed or repeated keys) sets *flag and the host sorts with digit passes
// over every varying byte instead.
constexpr int LT = 512, LCAP = 4096, LPT = LCAP / LT, RUN_MAX = 256, LSTEP = LCAP - RUN_MAX;

// the prefix digits (offsets o.x > o.y > ...; an offset < 0: no digit)
__device__ __forceinline__ uint32_t prefix3(uint32_t bs, uint64_t z, int4 o) {
  uint32_t p = 0;
  p = (p << 8) | (o.x >= 0 ? key_digit(bs, z, o.x) : 0u);
  p = (p << 8) | (o.y >= 0 ? key_digit(bs, z, o.y) : 0u);
  p = (p << 8) | (o.z >= 0 ? key_digit(bs, z, o.z) : 0u);
  p = (p << 8) | (o.w >= 0 ? key_digit(bs, z, o.w) : 0u);
  return p;
}

template <bool SH>
__global__ __launch_bounds__(LT) void k_sort_local(const uint8_t* __restrict__ sh_in, const uint16_t* __restrict__ bin_in,
                                                   const uint64_t* __restrict__ z_in, const uint32_t* __restrict__ perm_in,
                                                   uint8_t* __restrict__ sh_out, uint16_t* __restrict__ bin_out,
                                                   uint64_t* __restrict__ z_out, int64_t* __restrict__ perm_out,
                                                   int64_t n, int4 po, uint32_t* __restrict__ flag) {
  __shared__ uint64_t s_z[LCAP];
  __shared__ uint32_t s_bs[LCAP];
  __shared__ uint32_t s_run[LCAP];   // prefix; then run start (low 16) | at a run start, its end << 16
  __shared__ int64_t s_ab[2];
  __shared__ uint32_t s_wmax[LT / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  auto gbs = [&](int64_t r) -> uint32_t { return (uint32_t)bin_in[r] | (SH ? (uint32_t)sh_in[r] << 16 : 0u); };
  const int64_t ntile = (n + LSTEP - 1) / LSTEP;
  for (int64_t tk = blockIdx.x; tk < ntile; tk += gridDim.x) {   // block-uniform
    if (wave < 2) {   // waves 0 / 1: the first run start at or after p (none within RUN_MAX rows: flag)
      int64_t p = min(n, (tk + wave) * LSTEP);
      if (p > 0 && p < n) {
        const uint32_t pp = prefix3(gbs(p - 1), z_in[p - 1], po);
        int64_t found = -1;
        for (int c = 0; c <= RUN_MAX / 64 && found < 0; ++c) {   // wave-uniform
          const int64_t r = p + c * 64 + lane;
          const bool diff = r >= n || prefix3(gbs(r), z_in[r], po) != pp;
          const uint64_t bal = __ballot(diff);
          if (bal) found = p + c * 64 + __builtin_ctzll(bal);
        }
        p = (found < 0 || found - p > RUN_MAX) ? -1 : found;
        if (p < 0 && lane == 0) *flag = 1u;
      }
      if (lane == 0) s_ab[wave] = p;
    }
    __syncthreads();
    const int64_t a = s_ab[0], b = s_ab[1];
    __syncthreads();
    if (a < 0 || b < 0) continue;   // flagged: the host redoes the sort
    const int m = (int)(b - a);     // <= LSTEP + RUN_MAX = LCAP
    for (int i = t; i < m; i += LT) {
      const uint64_t zz = z_in[a + i];
      const uint32_t bb = gbs(a + i);
      s_z[i] = zz; s_bs[i] = bb; s_run[i] = prefix3(bb, zz, po);
    }
    __syncthreads();
    // run starts: a block max-scan of (row starts a run ? row : 0) over rows [LPT t, LPT t + LPT)
    uint32_t st[LPT];
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = LPT * t + k;
      if (i < m && (i == 0 || s_run[i] != s_run[i - 1])) run = (uint32_t)i;
      st[k] = run;
    }
    uint32_t x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x = max(x, y);
    }
    if (lane == 63) s_wmax[wave] = x;
    __syncthreads();
    uint32_t carry = 0;
    for (int w = 0; w < wave; ++w) carry = max(carry, s_wmax[w]);
    const uint32_t prev = __shfl_up(x, 1, 64);
    if (lane > 0) carry = max(carry, prev);
#pragma unroll
    for (int k = 0; k < LPT; ++k) st[k] = max(st[k], carry);
    __syncthreads();   // every prefix read before s_run is overwritten
#pragma unroll
    for (int k = 0; k < LPT; ++k)
      if (LPT * t + k < m) s_run[LPT * t + k] = st[k];
    __syncthreads();
    // a run's end, stored at its start: written by the next run's first row (or the tile's last row)
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = LPT * t + k;
      if (i < m && i > 0 && st[k] == (uint32_t)i) {
        const uint32_t ps = s_run[i - 1] & 0xffffu;
        s_run[ps] = ps | ((uint32_t)i << 16);
      }
      if (i == m - 1) s_run[st[k]] = st[k] | ((uint32_t)m << 16);
    }
    __syncthreads();
    for (int i = t; i < m; i += LT) {
      const int s0 = (int)(s_run[i] & 0xffffu), e0 = (int)(s_run[s0] >> 16);
      if (e0 - s0 > RUN_MAX) { *flag = 1u; continue; }
      const uint64_t zi = s_z[i];
      const uint32_t bi = s_bs[i];
      int r = 0;
      for (int j = s0; j < e0; ++j) {
        const uint32_t bj = s_bs[j];
        const uint64_t zj = s_z[j];
        r += (bj < bi) || (bj == bi && (zj < zi || (zj == zi && j < i)));
      }
      const int64_t dst = a + s0 + r;
      z_out[dst] = zi;
      bin_out[dst] = (uint16_t)bi;
      if (SH) sh_out[dst] = (uint8_t)(bi >> 16);
      perm_out[dst] = perm_in ? (int64_t)perm_in[a + i] : a + i;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(STPB) void k_widen_perm(const uint32_t* __restrict__ p32, int64_t n, int64_t* __restrict__ p64) {
  for (int64_t i = (int64_t)blockIdx.x * STPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * STPB) p64[i] = p32 ? p32[i] : i;
}

// ------------------------------------------------------------------ row-key bytes
// 256 rows per block: each thread writes its row's bytes into LDS, then the block's contiguous
// 256 * key_len bytes (a multiple of 16) leave with 16-B stores.
__global__ __launch_bounds__(STPB) void k_key_bytes(const uint8_t* __restrict__ sh, const int16_t* __restrict__ bin,
                                                    const int64_t* __restrict__ z, int64_t n, int klen,
                                                    uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t s[STPB * 11];
  const int64_t r0 = (int64_t)blockIdx.x * STPB;
  const int64_t i = r0 + threadIdx.x;
  if (i < n) {
    uint8_t* o = s + threadIdx.x * klen;
    int k = 0;
    if (klen == 11) o[k++] = sh[i];
    const uint16_t b = (uint16_t)bin[i];
    o[k++] = (uint8_t)(b >> 8);
    o[k++] = (uint8_t)b;
    const uint64_t zz = (uint64_t)z[i];
#pragma unroll
    for (int j = 7; j >= 0; --j) o[k++] = (uint8_t)(zz >> (8 * j));
  }
  __syncthreads();
  const int64_t rows = min((int64_t)STPB, n - r0);
  const int64_t bytes = rows * klen;
  uint8_t* dst = out + r0 * klen;
  if (rows == STPB && (((uintptr_t)dst) & 15u) == 0) {
    const uint4* s4 = (const uint4*)s;
    uint4* d4 = (uint4*)dst;
    for (int j = threadIdx.x; j < bytes / 16; j += STPB) d4[j] = s4[j];
  } else {
    for (int64_t j = threadIdx.x; j < bytes; j += STPB) dst[j] = s[j];
  }
}

}  // namespace gm

using namespace gm;

extern "C" {

int gm_z3_key_bytes(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n, uint8_t* out) {
  if (!ctx || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!bin || !z || !out) return GM_E_INVALID;
  const int klen = shard ? 11 : 10;
  hipLaunchKernelGGL(k_key_bytes, dim3((unsigned)((n + STPB - 1) / STPB)), dim3(STPB), 0, ctx->stream, shard, bin, z,
                     n, klen, out);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

int gm_sort_keys(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                 uint8_t* shard_out, int16_t* bin_out, int64_t* z_out, int64_t* perm_out) {
  if (!ctx || n < 0 || n > (int64_t)UINT32_MAX) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!bin || !z || !bin_out || !z_out || !perm_out || ((shard == nullptr) != (shard_out == nullptr)))
    return GM_E_INVALID;
  hipStream_t s = ctx->stream;
  const uint8_t* sh = shard;
  // 16-B z / 4-B bin / 2-B shard pair loads need aligned caller columns (the workspaces are)
  const bool user_vec = ((uintptr_t)z % 16) == 0 && ((uintptr_t)bin % 4) == 0 && (!sh || ((uintptr_t)sh % 2) == 0);
  const bool out_vec = ((uintptr_t)z_out % 16) == 0 && ((uintptr_t)bin_out % 4) == 0 &&
                       (!sh || ((uintptr_t)shard_out % 2) == 0);
  // which key bits vary (k_key_or_and): acc = OR z, OR bs, AND z, AND bs (bs = bin | shard << 16)
  unsigned long long* acc = (unsigned long long*)ctx->d_scratch;
  GM_HIP(hipMemsetAsync(acc, 0, 16, s));
  GM_HIP(hipMemsetAsync(acc + 2, 0xff, 16, s));
  GM_HIP(hipMemsetAsync(acc + 4, 0, 8, s));   // k_sort_local's flag
  hipLaunchKernelGGL(k_key_or_and, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(2048, (n / 2 + STPB - 1) / STPB))),
                     dim3(STPB), 0, s, sh, (const uint16_t*)bin, (const uint64_t*)z, n, acc, (int)user_vec);
  GM_CHECK_LAUNCH();
  unsigned long long hacc[4];
  GM_HIP(hipMemcpyAsync(hacc, acc, sizeof(hacc), hipMemcpyDeviceToHost, s));
  GM_HIP(hipStreamSynchronize(s));
  // LSD digit offsets: every byte on which some keys differ
  std::vector<int> lsd;
  for (int p = 0; p < NPASS; ++p) {
    if (p == 10 && !sh) continue;
    const uint64_t o = p < 8 ? hacc[0] >> (8 * p) : hacc[1] >> (8 * (p - 8));
    const uint64_t a = p < 8 ? hacc[2] >> (8 * p) : hacc[3] >> (8 * (p - 8));
    if (((o ^ a) & 255u) != 0) lsd.push_back(8 * p);
  }
  if (lsd.empty()) {  // every key equal: table order = input order
    if (sh) GM_HIP(hipMemcpyAsync(shard_out, sh, (size_t)n, hipMemcpyDeviceToDevice, s));
    GM_HIP(hipMemcpyAsync(bin_out, bin, (size_t)n * 2, hipMemcpyDeviceToDevice, s));
    GM_HIP(hipMemcpyAsync(z_out, z, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_widen_perm, dim3((unsigned)std::min<int64_t>(4096, (n + STPB - 1) / STPB)), dim3(STPB), 0, s,
                       nullptr, n, perm_out);
    GM_CHECK_LAUNCH();
    ctx->sort_last = 0;
    return GM_OK;
  }
  // prefix passes: digits each ending at the highest varying bit below the previous one (only constant
  // bits are skipped), ceil((log2 n + 3) / 8) of them (at most 4), when that is fewer than the
  // varying bytes
  const uint64_t vz = hacc[0] ^ hacc[2], vb = (hacc[1] ^ hacc[3]) & 0xffffffull;
  auto varying = [&](int bit) -> bool { return bit < 64 ? ((vz >> bit) & 1u) : ((vb >> (bit - 64)) & 1u); };
  int lg = 0;
  while (((int64_t)1 << lg) < n) ++lg;
  const int npre = std::min(4, (lg + 3 + 7) / 8);
  int pofs[4] = {-1, -1, -1, -1};
  int nfound = 0;
  {
    int bit = 87;
    for (int k = 0; k < npre; ++k) {
      while (bit >= 0 && !varying(bit)) --bit;
      if (bit < 0) break;
      pofs[k] = std::max(0, bit - 7);
      bit = pofs[k] - 1;
      ++nfound;
    }
  }
  const bool prefix_mode = ctx->sort_mode == 0 && (int)lsd.size() > npre && nfound == npre;
  // one resident wave of blocks: the scatter's LDS (~139 KiB) allows one 1024-thread block per CU
  const int resident = resident_blocks((const void*)k_sort_scatter<false, true>, ctx->device, BT, 1);
  const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(resident, (n + BTILE - 1) / BTILE));
  const int64_t per = ((n + nblk - 1) / nblk + BTILE - 1) / BTILE * BTILE;
  const int grid = (int)((n + per - 1) / per);
  // ping-pong: the user outputs and one temp set
  uint8_t* tsh = nullptr;
  uint16_t* tbin = nullptr;
  uint64_t* tz = nullptr;
  uint32_t *p0 = nullptr, *p1 = nullptr, *hist = nullptr;
  int64_t* hpart = nullptr;
  {  // context-owned workspace: z | perm 0 | perm 1 | bin | hist | shard, 16-B aligned pieces
    auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
    const size_t a_z = al((size_t)n * 8), a_p = al((size_t)n * 4), a_b = al((size_t)n * 2),
                 a_h = al((size_t)256 * grid * 4), a_s = sh ? al((size_t)n) : 0,
                 a_pt = al((size_t)scan_partials_len((int64_t)256 * grid) * 8);
    void* base = nullptr;
    int wrc = ctx_workspace(ctx, WS_SORT, a_z + 2 * a_p + a_b + a_h + a_pt + a_s, &base);
    if (wrc) return wrc;
    char* q = (char*)base;
    tz = (uint64_t*)q; q += a_z;
    p0 = (uint32_t*)q; q += a_p;
    p1 = (uint32_t*)q; q += a_p;
    tbin = (uint16_t*)q; q += a_b;
    hist = (uint32_t*)q; q += a_h;
    hpart = (int64_t*)q; q += a_pt;
    if (sh) tsh = (uint8_t*)q;
  }
  // digit passes at bit offsets `offs` (LSD order) from the caller's columns; the last pass lands in
  // the user outputs when `to_user_last`, else in the workspace (read by k_sort_local); `perm64`:
  // the last pass writes the 64-bit permutation
  const uint8_t *rsh = nullptr;
  const uint16_t* rbin = nullptr;
  const uint64_t* rz = nullptr;
  const uint32_t* rperm = nullptr;
  auto passes = [&](const std::vector<int>& offs, bool to_user_last) -> int {
    const int np = (int)offs.size();
    const uint8_t* ish = sh;
    const uint16_t* ibin = (const uint16_t*)bin;
    const uint64_t* iz = (const uint64_t*)z;
    const uint32_t* iperm = nullptr;
    for (int k = 0; k < np; ++k) {
      const bool to_user = ((np - 1 - k) % 2 == 0) == to_user_last;
      uint8_t* osh = sh ? (to_user ? shard_out : tsh) : nullptr;
      uint16_t* obin = to_user ? (uint16_t*)bin_out : tbin;
      uint64_t* oz = to_user ? (uint64_t*)z_out : tz;
      uint32_t* operm = (k % 2) ? p1 : p0;
      // pass 0 reads the caller's columns, a later pass reads the caller's outputs or the workspace
      const int vec = k == 0 ? (int)user_vec : (ibin == (const uint16_t*)bin_out ? (int)out_vec : 1);
      hipLaunchKernelGGL(k_sort_hist, dim3(grid), dim3(HT), 0, s, ish, ibin, iz, n, per, offs[k], hist, vec);
      launch_excl_scan(s, hist, (int64_t)256 * grid, hist, hpart, (int64_t*)nullptr);
      const bool last64 = to_user_last && k == np - 1;   // the last pass writes the 64-bit permutation itself
      auto scatter = sh ? (iperm ? k_sort_scatter<true, true> : k_sort_scatter<true, false>)
                        : (iperm ? k_sort_scatter<false, true> : k_sort_scatter<false, false>);
      hipLaunchKernelGGL(scatter, dim3(grid), dim3(BT), 0, s, ish, ibin, iz, iperm, osh, obin, oz,
                         last64 ? nullptr : operm, last64 ? perm_out : nullptr, n, per, offs[k], hist, vec);
      if (hipGetLastError() != hipSuccess) return hip_fail(hipErrorLaunchFailure, "k_sort_scatter");
      ish = osh; ibin = obin; iz = oz; iperm = operm;
    }
    rsh = ish; rbin = ibin; rz = iz; rperm = iperm;
    return GM_OK;
  };
  if (prefix_mode) {
    std::vector<int> offs(pofs, pofs + npre);
    std::reverse(offs.begin(), offs.end());   // LSD order: lowest digit first
    int rc = passes(offs, false);
    if (rc) return rc;
    const int4 po = make_int4(pofs[0], pofs[1], pofs[2], pofs[3]);
    const int lgrid = resident_blocks((const void*)k_sort_local<false>, ctx->device, LT, 2);
    if (sh)
      hipLaunchKernelGGL(k_sort_local<true>, dim3(lgrid), dim3(LT), 0, s, rsh, rbin, rz, rperm, shard_out,
                         (uint16_t*)bin_out, (uint64_t*)z_out, perm_out, n, po, (uint32_t*)(acc + 4));
    else
      hipLaunchKernelGGL(k_sort_local<false>, dim3(lgrid), dim3(LT), 0, s, rsh, rbin, rz, rperm, nullptr,
                         (uint16_t*)bin_out, (uint64_t*)z_out, perm_out, n, po, (uint32_t*)(acc + 4));
    GM_CHECK_LAUNCH();
    uint32_t flag = 0;
    GM_HIP(hipMemcpyAsync(&flag, acc + 4, 4, hipMemcpyDeviceToHost, s));
    GM_HIP(hipStreamSynchronize(s));
    if (!flag) {
      ctx->sort_last = 256 + npre;
      return GM_OK;
    }
    // a run of equal prefixes longer than RUN_MAX: digit passes over every varying byte
  }
  ctx->sort_last = (int64_t)lsd.size() + (prefix_mode ? npre : 0);   // (a failed prefix attempt included)
  return passes(lsd, true);
}

}  // extern "C"
