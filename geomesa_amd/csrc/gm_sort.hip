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
//                         AND), a second counts every pass's digits at once (k_sort_count).  Then
//                         one-sweep digit passes (digits of <= 9 bits, k_sort_pass): 8192-row tiles
//                         taken in order, ranked in LDS (wave ballots rank equal digits), each tile's
//                         digit offsets found by a decoupled look-back over the tiles before it (8-B
//                         {count, tag} granules), and the tile leaves as digit runs of 16-B records
//                         {z, row, bs} (bs = bin | shard << sq, squeeze_bs).  The passes order the rows by the top
//                         ~log2(n) - 1 varying bits (three 9-bit digits at 250M rows); k_local_bounds
//                         cuts the result into ~2048-row tiles at run starts and k_sort_local ranks
//                         every run of equal prefixes (a few rows) by full key in LDS and writes the
//                         user columns.  A run longer than 256 rows (skewed keys) sends the
//                         call to 8-bit digit passes over every varying byte (LSD, the same kernels),
//                         which is also GM_PARAM_SORT_MODE 1.
// The range scan over a sorted table (gm_key_range_scan) lives with the other row-filter scans in
// gm_filter.hip.
#include <string.h>

#include <algorithm>
#include <vector>

#include "gm_scan.hpp"

namespace gm {

constexpr int STPB = 256;               // key-byte threads per block
constexpr int NPASS = 11;               // digit positions: z bytes 0..7, bin bytes 0..1, shard
constexpr int MAXTAG = 16;              // pass tags per call: prefix passes + a fallback's digit passes

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

// a row in flight between passes: {z lo, z hi, input row, bs} (bs = bin | shard << sq, squeeze_bs)
__device__ __forceinline__ uint64_t rec_z(uint4 r) { return (uint64_t)r.x | ((uint64_t)r.y << 32); }
__device__ __forceinline__ uint4 make_rec(uint64_t z, uint32_t row, uint32_t bs) {
  return make_uint4((uint32_t)z, (uint32_t)(z >> 32), row, bs);
}

// With a shard byte, the sort's key packs it right above bin's highest varying bit: bs = bin low bits |
// shard << sq (sq = that bit + 1, 16 without a shard).  The bits of bin above it are the same in every
// key (binhi), so this order is the (shard, bin) order, and the key's varying bits are contiguous: the
// prefix digits cover shard and bin together instead of a 9-bit digit spanning bin's constant top bits
// (with 4 shards and weekly bins that digit held 2 varying bits of 9, the runs of equal prefixes grew to
// ~128 rows and the sort took 31.5 ms per 250M rows instead of ~10.5).
__device__ __forceinline__ uint32_t squeeze_bs(uint32_t b, int sq) { return (b & ((1u << sq) - 1u)) | ((b >> 16) << sq); }
__device__ __forceinline__ uint16_t bs_bin(uint32_t w, int sq, uint32_t binhi) {
  return (uint16_t)((w & ((1u << sq) - 1u)) | binhi);
}
__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// The caller's columns, read two rows per lane (16-B z, 4-B bin, 2-B shard loads) when `vec` (aligned
// columns) and both rows exist, else row by row.  bs = bin | shard << 16.
struct KeyCols {
  const uint8_t* sh;
  const uint16_t* bin;
  const uint64_t* z;
};
template <bool SH>
__device__ __forceinline__ void load_pair(const KeyCols& c, int64_t i, int64_t n, bool vec, uint64_t& z0, uint64_t& z1,
                                          uint32_t& bs0, uint32_t& bs1) {
  if (vec && i + 1 < n) {
    const ulonglong2 zz = *(const ulonglong2*)(c.z + i);
    const uint32_t bb = *(const uint32_t*)(c.bin + i);
    z0 = zz.x; z1 = zz.y;
    bs0 = bb & 0xffffu; bs1 = bb >> 16;
    if (SH) {
      const uint32_t ss = *(const uint16_t*)(c.sh + i);
      bs0 |= (ss & 0xffu) << 16; bs1 |= (ss >> 8) << 16;
    }
  } else {
    z0 = z1 = 0; bs0 = bs1 = 0;
    if (i < n) { z0 = c.z[i]; bs0 = (uint32_t)c.bin[i] | (SH ? (uint32_t)c.sh[i] << 16 : 0u); }
    if (i + 1 < n) { z1 = c.z[i + 1]; bs1 = (uint32_t)c.bin[i + 1] | (SH ? (uint32_t)c.sh[i + 1] << 16 : 0u); }
  }
}

// which digit passes carry information: the OR and the AND of every key column (a digit on which
// OR == AND is the same for every key, so its pass would be the identity and is skipped).
// acc[0] = OR z, acc[1] = OR bs, acc[2] = AND z, acc[3] = AND bs.  Four pairs per lane in flight.
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
// f(z, bs) over every row of the caller's columns, one wave per 512-row chunk.  With 16-B aligned
// columns (`wide`) every load is one contiguous 1 KiB per wave instruction: z as 16-B pairs (rows
// 128 u + 2 lane, + 1), bin as 8 rows per lane and the shard byte as 16 per lane, staged through the
// wave's LDS slice so each lane meets the bins of its z rows (narrow per-lane loads stream at about
// half the 16-B rate on gfx950); other chunks go row by row.
constexpr int RCH = 512;   // rows per wave chunk
template <bool SH, int NWAVE, class F>
__device__ __forceinline__ void for_rows(const KeyCols& c, int64_t n, int wide, F f) {
  __shared__ __attribute__((aligned(16))) uint16_t s_b[NWAVE][RCH];
  __shared__ __attribute__((aligned(16))) uint8_t s_s[NWAVE][SH ? RCH : 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t nchunk = (n + RCH - 1) / RCH, stride = (int64_t)gridDim.x * NWAVE;
  for (int64_t ch = (int64_t)blockIdx.x * NWAVE + wave; ch < nchunk; ch += stride) {   // wave-uniform
    const int64_t r0 = ch * RCH;
    if (wide && r0 + RCH <= n) {
      ulonglong2 zz[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) zz[u] = *(const ulonglong2*)(c.z + r0 + 128 * u + 2 * lane);
      *(uint4*)&s_b[wave][8 * lane] = *(const uint4*)(c.bin + r0 + 8 * lane);
      if (SH && lane < RCH / 16) *(uint4*)&s_s[wave][16 * lane] = *(const uint4*)(c.sh + r0 + 16 * lane);
      wave_lds_sync();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int j = 128 * u + 2 * lane;
        f(zz[u].x, (uint32_t)s_b[wave][j] | (SH ? (uint32_t)s_s[wave][j] << 16 : 0u));
        f(zz[u].y, (uint32_t)s_b[wave][j + 1] | (SH ? (uint32_t)s_s[wave][j + 1] << 16 : 0u));
      }
      wave_lds_sync();   // the slice is free for the next chunk
    } else {
      for (int64_t r = r0 + lane; r < min(n, r0 + RCH); r += 64)
        f(c.z[r], (uint32_t)c.bin[r] | (SH ? (uint32_t)c.sh[r] << 16 : 0u));
    }
  }
}

// The OR / AND of a strided sample of the keys (65,536 rows, the last row included): the host plans the
// digits from it and k_sort_count counts them in the same read that takes the exact OR / AND; a plan
// that the exact bits change is counted again (GM_PARAM_SORT_LAST reports the path either way)
constexpr int SAMPLE = 65536;
template <bool SH>
__global__ __launch_bounds__(256) void k_key_or_and_sample(KeyCols c, int64_t n, unsigned long long* __restrict__ acc) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t step = n > SAMPLE ? n / SAMPLE : 1;
  uint64_t zo = 0, za = ~0ull, bo = 0, ba = ~0ull;
  auto take = [&](int64_t r) {
    const uint64_t z = c.z[r];
    const uint32_t b = (uint32_t)c.bin[r] | (SH ? (uint32_t)c.sh[r] << 16 : 0u);
    zo |= z; za &= z; bo |= b; ba &= b;
  };
  if (i < SAMPLE && i * step < n) take(i * step);
  if (i == 0) take(n - 1);
  __shared__ uint64_t s_oa[4][4];
  zo = wave_or(zo); za = wave_and(za); bo = wave_or(bo); ba = wave_and(ba);
  if ((threadIdx.x & 63) == 0) {
    uint64_t* e = s_oa[threadIdx.x >> 6];
    e[0] = zo; e[1] = bo; e[2] = za; e[3] = ba;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int j = threadIdx.x;
    uint64_t v = s_oa[0][j];
    for (int w = 1; w < 4; ++w) v = j < 2 ? (v | s_oa[w][j]) : (v & s_oa[w][j]);
    if (j < 2) atomicOr(&acc[j], (unsigned long long)v);
    else atomicAnd(&acc[j], (unsigned long long)v);
  }
}

// Every pass's digit counts in one read: counts[base_k + d] = rows whose digit k (bits [off_k, off_k +
// w_k) of K) is d, base_k = k * 512.  Four LDS copies of the counters (by wave) cut the atomic
// collisions.  ORAND: the same read also takes the exact OR / AND of the key columns into
// acc[0..3] = OR z, OR bs, AND z, AND bs (bs = bin | shard << 16).
constexpr int WMAX = 9;                 // widest digit: 512 buckets
constexpr int NB_MAX = 1 << WMAX;
struct DigitOffs {
  int off[NPASS];
  int w[NPASS];
  int np;
};
__device__ __forceinline__ uint32_t key_digit_w(uint32_t bs, uint64_t z, int off, int w) {
  return key_bits(bs, z, off) & ((1u << w) - 1u);
}
constexpr int CNT_LDS = 2816;           // 11 byte digits x 256, or 4 prefix digits x 512 (<= 2048)
constexpr int CT = 1024;   // count threads per block
template <bool SH, bool ORAND>
__global__ __launch_bounds__(CT) void k_sort_count(KeyCols c, int64_t n, DigitOffs o, uint32_t* __restrict__ counts, int wide,
                                                   unsigned long long* __restrict__ acc, int sq) {
  __shared__ uint32_t h[4][CNT_LDS];
  const int copy = (threadIdx.x >> 6) & 3;
  for (int i = threadIdx.x; i < 4 * CNT_LDS; i += CT) (&h[0][0])[i] = 0u;
  __syncthreads();
  uint64_t zo = 0, za = ~0ull, bo = 0, ba = ~0ull;
  for_rows<SH, CT / 64>(c, n, wide, [&](uint64_t z, uint32_t b) {
    if (ORAND) { zo |= z; za &= z; bo |= b; ba &= b; }   // of the caller's bs (bin | shard << 16)
    const uint32_t bk_s = SH ? squeeze_bs(b, sq) : b;
    for (int k = 0, bk = 0; k < o.np; bk += 1 << o.w[k], ++k)
      atomicAdd(&h[copy][bk + key_digit_w(bk_s, z, o.off[k], o.w[k])], 1u);
  });
  __shared__ uint64_t s_oa[ORAND ? CT / 64 : 1][4];
  if (ORAND) {   // per wave, then one device atomic per value per block (not per wave: same 4 addresses)
    zo = wave_or(zo); za = wave_and(za); bo = wave_or(bo); ba = wave_and(ba);
    if ((threadIdx.x & 63) == 0) {
      uint64_t* e = s_oa[threadIdx.x >> 6];
      e[0] = zo; e[1] = bo; e[2] = za; e[3] = ba;
    }
  }
  __syncthreads();
  if (ORAND && threadIdx.x < 4) {
    const int j = threadIdx.x;
    uint64_t v = s_oa[0][j];
    for (int w = 1; w < CT / 64; ++w) v = j < 2 ? (v | s_oa[w][j]) : (v & s_oa[w][j]);
    if (j < 2) atomicOr(&acc[j], (unsigned long long)v);
    else atomicAnd(&acc[j], (unsigned long long)v);
  }
  for (int k = 0, bk = 0; k < o.np; bk += 1 << o.w[k], ++k)
    for (int d = threadIdx.x; d < (1 << o.w[k]); d += CT) {
      const int i = bk + d;
      const uint32_t v = h[0][i] + h[1][i] + h[2][i] + h[3][i];
      if (v) atomicAdd(&counts[k * NB_MAX + d], v);
    }
}

// One-sweep digit pass over a digit of w <= 9 bits.  Block b takes tile k (the next in a counter, so
// every lower tile is already running) of 8192 rows; wave w owns rows [512 w, 512 w + 512) of it and
// reads them in 4 slots of 128 rows, 2 per lane.  Within a slot, lanes holding the same digit find each
// other with 2 w ballots (w digit bits x even / odd row); a per-wave LDS counter per digit turns slot
// ranks into wave ranks, a scan over the waves into tile ranks, so a row's place in the tile is
// (digit, wave, slot, lane, even / odd) = stable.  The tile's digit offsets in the output are the
// digit's global start plus its rows in every lower tile: thread d publishes digit d's tile count as
// soon as the tile is ranked ({count, AGG} granule, one 8-B write-through store), then walks back over
// the lower tiles' granules, adding counts until it meets an inclusive prefix (PRE), and publishes its
// own (decoupled look-back).  The tile is reordered in LDS meanwhile and leaves as digit runs of 16-B
// records.  Granule tags carry the pass (tag) so no pass reads another's; the status array is cleared
// once per call.  1024-thread blocks over 8192-row tiles (LDS ~148 KB: one block, 16 waves, per CU):
// 10.84-10.86 -> 10.48-10.51 ms per 250M-row sort against 512 threads / 4096 rows at two blocks per CU
// once the tile's loads were all in flight together (profiles/r5/sort_tile_shape_ab.txt; 768 threads
// 11.97-11.99, 1024 x 2048 rows 13.75-13.77, 1024 x 6144 11.63-11.67, 512 x 8192 11.30-11.35).
#ifndef GM_SORT_PSLOT
#define GM_SORT_PSLOT 4
#endif
#ifndef GM_SORT_PT
#define GM_SORT_PT 1024
#endif
constexpr int PT = GM_SORT_PT, PW = PT / 64, PSLOT = GM_SORT_PSLOT, PTILE = PT * 2 * PSLOT;   // 8192 rows per tile
static_assert(PT >= NB_MAX, "one thread per digit");
constexpr uint64_t GR_VAL = (1ull << 48) - 1;
#ifndef GM_SORT_LB
#define GM_SORT_LB 4
#endif
constexpr int LB = GM_SORT_LB;   // look-back granules per round trip
#ifndef GM_SORT_SPLIT
#define GM_SORT_SPLIT 1
#endif
#ifndef GM_SORT_LDSMATCH
#define GM_SORT_LDSMATCH 1
#endif

struct PassArgs {
  KeyCols in;             // the caller's columns (first pass) ...
  const uint4* rec_in;    // ... or the previous pass's records
  uint8_t* sh_out;        // the caller's outputs (last pass) ...
  uint16_t* bin_out;
  uint64_t* z_out;
  int64_t* perm_out;
  uint4* rec_out;         // ... or records
  int64_t n;
  int off, w;             // digit: bits [off, off + w) of K
  uint32_t tag;           // 1..MAXTAG
  const uint32_t* counts;           // this pass's 2^w digit counts
  unsigned long long* status;       // ntiles x 2^w granules
  unsigned int* ctr;                // this pass's tile counter
  int vec;
  int sq;                 // the shard's place in the records' bs (squeeze_bs) ...
  uint32_t binhi;         // ... and bin's constant bits above it
};

template <bool IN_REC, bool OUT_USER, bool SH>
__global__ __launch_bounds__(PT) void k_sort_pass(PassArgs a) {
  __shared__ uint4 s_rec[PTILE];
  __shared__ uint16_t s_wcnt[PW][NB_MAX];   // per wave: rows of each digit so far (then: wave offsets)
  __shared__ uint32_t s_dstart[NB_MAX];     // the digit's first slot in the tile
  __shared__ uint32_t s_gpos[NB_MAX];       // output row of tile slot q = s_gpos[d] + q (mod 2^32)
  __shared__ uint32_t s_wsum[2][PW];
  __shared__ uint32_t s_tile;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int w = a.w, nb = 1 << w;
  // this pass's global count of digit t, loaded before anything waits (used after the ranking)
  const uint32_t cg_early = t < nb ? a.counts[t] : 0u;
  if (t == 0) s_tile = atomicAdd(a.ctr, 1u);
  for (int i = t; i < PW * NB_MAX / 2; i += PT) ((uint32_t*)&s_wcnt[0][0])[i] = 0u;
  __syncthreads();
  const int64_t tile = s_tile, t0 = tile * PTILE, n = a.n;
#if GM_SORT_SPLIT
  // this lane's rows: slot k of wave w holds rows r = t0 + 512 w + 128 k + lane (A) and r + 64 (B), so
  // in input order a slot is its 64 A rows, then its 64 B rows, and each half ranks like one row per
  // lane: 9 ballots and one mask per row.  (Round 5's pairs (2 lane, 2 lane + 1) interleave the halves
  // and needed four cross masks per pair: ~80 instead of ~45 VALU per row in the ranking.)
  uint4 rv[PSLOT][2];
  const bool full = t0 + PTILE <= n;   // every tile but the last (uniform)
  const bool vec = a.vec && full;
  if (IN_REC && full) {
    // a full tile's loads are unconditional, so the compiler counts them: all 2 * PSLOT are in flight
    // before the first wait
#pragma unroll
    for (int k = 0; k < PSLOT; ++k) {
      const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + lane;
      rv[k][0] = a.rec_in[i];
      rv[k][1] = a.rec_in[i + 64];
    }
  } else if (!IN_REC && vec) {   // the same for the first pass's column loads
#pragma unroll
    for (int k = 0; k < PSLOT; ++k)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 64 * e + lane;
        uint32_t b = (uint32_t)a.in.bin[i];
        if (SH) b = squeeze_bs(b | (uint32_t)a.in.sh[i] << 16, a.sq);
        rv[k][e] = make_rec(a.in.z[i], (uint32_t)i, b);
      }
  } else {
#pragma unroll
    for (int k = 0; k < PSLOT; ++k)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 64 * e + lane;
        if (IN_REC) {
          rv[k][e] = i < n ? a.rec_in[i] : make_uint4(0u, 0u, 0u, 0u);
        } else {
          uint32_t b = i < n ? (uint32_t)a.in.bin[i] | (SH ? (uint32_t)a.in.sh[i] << 16 : 0u) : 0u;
          if (SH) b = squeeze_bs(b, a.sq);
          rv[k][e] = make_rec(i < n ? a.in.z[i] : 0ull, (uint32_t)i, b);
        }
      }
  }
  const uint64_t lt = lanemask_lt();
  uint32_t rd[PSLOT][2];   // wave rank | digit << 16; rank 0xffff = no row
#if GM_SORT_LDSMATCH
  // lanes sharing a digit found through LDS instead of 9 ballot rounds: each row ORs its lane bit into
  // its digit's 64-bit slot, reads the slot back, and clears it.  The slots (512 per wave, 64 KB) alias
  // s_rec, which is written only after the ranking's barrier.
  uint64_t* mslot = (uint64_t*)s_rec + wave * NB_MAX;
  for (int j = lane; j < NB_MAX; j += 64) mslot[j] = 0ull;
  wave_lds_sync();
#endif
#pragma unroll
  for (int k = 0; k < PSLOT; ++k)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 64 * e + lane;
      const bool ok = i < n;
      const uint32_t d = key_digit_w(rv[k][e].w, rec_z(rv[k][e]), a.off, w);
#if GM_SORT_LDSMATCH
      if (ok) atomicOr((unsigned long long*)&mslot[d], 1ull << lane);
      wave_lds_sync();
      const uint64_t m = ok ? mslot[d] : 0ull;   // lanes of this half whose row holds my row's digit
      wave_lds_sync();
      if (ok) mslot[d] = 0ull;
#else
      uint64_t m = __ballot(ok);   // lanes of this half whose row holds my row's digit
#pragma unroll
      for (int bit = 0; bit < WMAX; ++bit) {   // bits at or above w are 0 in every digit: no-op rounds
        const uint64_t bb = __ballot((d >> bit) & 1u);
        m &= ((d >> bit) & 1u) ? bb : ~bb;
      }
#endif
      const int r = __popcll(m & lt);
      // the wave's counter: read before this half's increment, then the first row of each digit adds
      const uint32_t c = s_wcnt[wave][d];
      rd[k][e] = (ok ? c + r : 0xffffu) | (d << 16);
      __builtin_amdgcn_wave_barrier();
      if (ok && r == 0) s_wcnt[wave][d] = (uint16_t)(c + __popcll(m));
      __builtin_amdgcn_wave_barrier();
    }
#else
  // this lane's rows
  uint4 rv[PSLOT][2];
  const bool full = t0 + PTILE <= n;   // every tile but the last (uniform)
  const bool vec = a.vec && full;
  if (IN_REC && full) {
    // a full tile's loads are unconditional, so the compiler counts them: all 2 * PSLOT are in flight
    // before the first wait.  (Under the per-row `i < n` selects each load sat in its own branch and
    // was waited for before the next one was issued: one load in flight per lane.)
#pragma unroll
    for (int k = 0; k < PSLOT; ++k) {
      const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 2 * lane;
      rv[k][0] = a.rec_in[i];
      rv[k][1] = a.rec_in[i + 1];
    }
  } else if (!IN_REC && vec) {   // the same for the first pass's column loads
#pragma unroll
    for (int k = 0; k < PSLOT; ++k) {
      const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 2 * lane;
      const ulonglong2 zz = *(const ulonglong2*)(a.in.z + i);
      uint32_t bb = *(const uint32_t*)(a.in.bin + i);
      uint32_t b0 = bb & 0xffffu, b1 = bb >> 16;
      if (SH) {
        const uint32_t ss = *(const uint16_t*)(a.in.sh + i);
        b0 = squeeze_bs(b0 | (ss & 0xffu) << 16, a.sq); b1 = squeeze_bs(b1 | (ss >> 8) << 16, a.sq);
      }
      rv[k][0] = make_rec(zz.x, (uint32_t)i, b0);
      rv[k][1] = make_rec(zz.y, (uint32_t)(i + 1), b1);
    }
  } else {
#pragma unroll
    for (int k = 0; k < PSLOT; ++k) {
      const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 2 * lane;
      if (IN_REC) {
        rv[k][0] = i < n ? a.rec_in[i] : make_uint4(0u, 0u, 0u, 0u);
        rv[k][1] = i + 1 < n ? a.rec_in[i + 1] : make_uint4(0u, 0u, 0u, 0u);
      } else {
        uint64_t z0, z1;
        uint32_t b0, b1;
        load_pair<SH>(a.in, i, n, vec, z0, z1, b0, b1);
        if (SH) { b0 = squeeze_bs(b0, a.sq); b1 = squeeze_bs(b1, a.sq); }
        rv[k][0] = make_rec(z0, (uint32_t)i, b0);
        rv[k][1] = make_rec(z1, (uint32_t)(i + 1), b1);
      }
    }
  }
  const uint64_t lt = lanemask_lt();
  uint32_t rd[PSLOT][2];   // wave rank | digit << 16; rank 0xffff = no row
#pragma unroll
  for (int k = 0; k < PSLOT; ++k) {
    const int64_t i = t0 + wave * (2 * 64 * PSLOT) + k * 128 + 2 * lane;
    const bool ok0 = i < n, ok1 = i + 1 < n;
    const uint32_t d0 = key_digit_w(rv[k][0].w, rec_z(rv[k][0]), a.off, w);
    const uint32_t d1 = key_digit_w(rv[k][1].w, rec_z(rv[k][1]), a.off, w);
    // masks of lanes whose even / odd row holds my even / odd row's digit
    uint64_t m00 = __ballot(ok0), m01 = __ballot(ok1);
    uint64_t m10 = m00, m11 = m01;
#pragma unroll
    for (int bit = 0; bit < WMAX; ++bit) {
      if (bit < w) {   // wave-uniform
        const uint64_t b0 = __ballot((d0 >> bit) & 1u), b1 = __ballot((d1 >> bit) & 1u);
        m00 &= ((d0 >> bit) & 1u) ? b0 : ~b0;
        m01 &= ((d0 >> bit) & 1u) ? b1 : ~b1;
        m10 &= ((d1 >> bit) & 1u) ? b0 : ~b0;
        m11 &= ((d1 >> bit) & 1u) ? b1 : ~b1;
      }
    }
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
#endif
  __syncthreads();
  // thread t owns digit t (t < nb): wave offsets, the tile total, scans of totals and global counts
  uint32_t tot = 0, xt = 0, xb = 0, cg = 0;
  const bool own = t < nb;
  if (own) {
#pragma unroll
    for (int v = 0; v < PW; ++v) {
      const uint32_t c = s_wcnt[v][t];
      s_wcnt[v][t] = (uint16_t)tot;
      tot += c;
    }
    // the tile's count for this digit, published before anything else
    const uint64_t g0 = ((uint64_t)(2 * a.tag + (tile == 0 ? 1 : 0)) << 48) | tot;
    __hip_atomic_store(a.status + tile * nb + t, g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    cg = cg_early;
  }
  xt = tot; xb = cg;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(xt, o, 64), yb = __shfl_up(xb, o, 64);
    if (lane >= o) { xt += y; xb += yb; }
  }
  if (lane == 63) { s_wsum[0][wave] = xt; s_wsum[1][wave] = xb; }
  __syncthreads();
  uint32_t dstart = 0, gbase = 0;
  if (own) {
    uint32_t pt = 0, pb = 0;
    for (int v = 0; v < wave; ++v) { pt += s_wsum[0][v]; pb += s_wsum[1][v]; }
    dstart = pt + xt - tot;
    gbase = pb + xb - cg;
    s_dstart[t] = dstart;
  }
  __syncthreads();
  // the tile reordered by digit in LDS
#pragma unroll
  for (int k = 0; k < PSLOT; ++k) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const uint32_t r = rd[k][e] & 0xffffu, d = rd[k][e] >> 16;
      if (r == 0xffffu) continue;
      s_rec[s_dstart[d] + s_wcnt[wave][d] + r] = rv[k][e];
    }
  }
  if (own) {   // look-back: the digit's rows in every lower tile
    uint64_t excl = 0;
    if (tile > 0) {
      const uint64_t tag_agg = 2 * a.tag, tag_pre = 2 * a.tag + 1;
      int64_t p = tile - 1;
      // LB granules (tiles p, p - 1, ..., p - LB + 1) per round trip, all loads in flight together:
      // the walk adds aggregates up to the first inclusive prefix, or re-polls from the first
      // granule not yet published.  Tile 0 always publishes a prefix, so no walk passes below it.
      for (;;) {
        uint64_t v[LB];
#pragma unroll
        for (int i = 0; i < LB; ++i)
          v[i] = p - i >= 0 ? __hip_atomic_load(a.status + (p - i) * nb + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : 0ull;
        int i = 0;
        bool done = false;
        for (; i < LB; ++i) {
          const uint64_t tg = v[i] >> 48;
          if (tg == tag_pre) { excl += v[i] & GR_VAL; done = true; break; }
          if (tg != tag_agg) break;
          excl += v[i] & GR_VAL;
        }
        if (done) break;
        p -= i;
        if (i < LB) __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(a.status + tile * nb + t, ((uint64_t)(2 * a.tag + 1) << 48) | (excl + tot),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_gpos[t] = gbase + (uint32_t)excl - dstart;   // mod 2^32: every output row is < n <= 2^32 - 1
  }
  __syncthreads();
  const int cnt = (int)min((int64_t)PTILE, n - t0);
  for (int q = t; q < cnt; q += PT) {
    const uint4 r = s_rec[q];
    const int64_t g = (int64_t)(uint32_t)(s_gpos[key_digit_w(r.w, rec_z(r), a.off, w)] + (uint32_t)q);
    if (OUT_USER) {
      a.z_out[g] = rec_z(r);
      a.bin_out[g] = SH ? bs_bin(r.w, a.sq, a.binhi) : (uint16_t)r.w;
      if (SH) a.sh_out[g] = (uint8_t)(r.w >> a.sq);
      a.perm_out[g] = (int64_t)r.z;
    } else {
      a.rec_out[g] = r;
    }
  }
}

// Final placement after the prefix passes: the digit passes at bit offsets o1 > o2 > ... (each digit
// ends at a varying bit, and only constant bits lie between them) leave the rows grouped, stably, by
// P = digit(o1) : digit(o2) : ... -- the key's top varying bits, ~log2(n) - 1 of them, so that runs
// of equal P are short (Poisson(n / 2^bits) for uniform keys, 2 rows on average).  Tile k covers the
// runs of equal P that start in [k LSTEP, (k + 1) LSTEP); its rows are staged in LDS, a block scan
// marks each row's run (start, and at the start its end), each row counts the rows of its run with a
// smaller key (ties by position: stable) and goes to run start + rank: O(run length) LDS reads per
// row.  A run longer than RUN_MAX rows (skewed or repeated keys) sets *flag and the host sorts with
// digit passes over every varying byte instead.
#ifndef GM_SORT_LCAP
#define GM_SORT_LCAP 2048
#endif
#ifndef GM_SORT_LT
#define GM_SORT_LT 512
#endif
constexpr int LT = GM_SORT_LT, LCAP = GM_SORT_LCAP, LPT = LCAP / LT, RUN_MAX = 256, LSTEP = LCAP - RUN_MAX;

// the prefix digits of width w (offsets o.x > o.y > ...; an offset < 0: no digit, and every later
// offset is < 0 too): npre * w <= 32 bits (gm_sort_keys), so the digits that exist are shifted in and
// the absent ones are not -- a shift per absent digit would push the first digit's top bits out of the
// word and merge distinct prefixes into one run
__device__ __forceinline__ uint32_t prefix4(uint32_t bs, uint64_t z, int4 o, int w) {
  uint32_t p = o.x >= 0 ? key_digit_w(bs, z, o.x, w) : 0u;
  if (o.y >= 0) p = (p << w) | key_digit_w(bs, z, o.y, w);
  if (o.z >= 0) p = (p << w) | key_digit_w(bs, z, o.z, w);
  if (o.w >= 0) p = (p << w) | key_digit_w(bs, z, o.w, w);
  return p;
}

// the local tiles' bounds: bounds[k] = the first run start at or after k LSTEP (0 and n at the ends;
// -1 and the flag when no run starts within RUN_MAX rows), one wave per bound, so that k_sort_local
// reads its next tile's bounds while it ranks the current one
__global__ __launch_bounds__(256) void k_local_bounds(const uint4* __restrict__ rec_in, int64_t n, int4 po, int pw,
                                                      int64_t* __restrict__ bounds, uint32_t* __restrict__ flag) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t ntile = (n + LSTEP - 1) / LSTEP;
  if (k > ntile) return;   // wave-uniform
  int64_t p = min(n, k * LSTEP);
  if (p > 0 && p < n) {
    const uint4 v0 = rec_in[p - 1];
    const uint32_t pp = prefix4(v0.w, rec_z(v0), po, pw);
    int64_t found = -1;
    for (int c = 0; c <= RUN_MAX / 64 && found < 0; ++c) {   // wave-uniform
      const int64_t r = p + c * 64 + lane;
      bool diff = r >= n;
      if (!diff) { const uint4 v = rec_in[r]; diff = prefix4(v.w, rec_z(v), po, pw) != pp; }
      const uint64_t bal = __ballot(diff);
      if (bal) found = p + c * 64 + __builtin_ctzll(bal);
    }
    p = (found < 0 || found - p > RUN_MAX) ? -1 : found;
    if (p < 0 && lane == 0) *flag = 1u;
  }
  if (lane == 0) bounds[k] = p;
}

// waves per SIMD: 8 = four resident 512-thread blocks per CU (64 VGPRs, no spills; the tiles' LDS is
// 32 KB each): 10.42-10.44 -> 10.22-10.25 ms per sort over the compiler's 75 VGPRs / three blocks;
// loading the next tile while ranking the current one instead: 11.61-11.66 ms
// (profiles/r5/sort_local_occupancy_ab.txt)
#ifndef GM_SORT_LOCAL_WPE
#define GM_SORT_LOCAL_WPE 8
#endif
template <bool SH>
__global__ __launch_bounds__(LT) __attribute__((amdgpu_waves_per_eu(GM_SORT_LOCAL_WPE))) void k_sort_local(
    const uint4* __restrict__ rec_in, uint8_t* __restrict__ sh_out, uint16_t* __restrict__ bin_out,
    uint64_t* __restrict__ z_out, int64_t* __restrict__ perm_out, int64_t n, int4 po, int pw,
    uint32_t* __restrict__ flag, const int64_t* __restrict__ bounds, int sq, uint32_t binhi) {
  __shared__ uint64_t s_z[LCAP];
  __shared__ uint32_t s_bs[LCAP];
  __shared__ uint32_t s_run[LCAP];   // prefix; then run start (low 16) | at a run start, its end << 16
  __shared__ uint32_t s_wmax[LT / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t ntile = (n + LSTEP - 1) / LSTEP;
  int64_t an = -1, bn = -1;   // the next tile's bounds (uniform: scalar loads, one tile ahead)
  if ((int64_t)blockIdx.x < ntile) { an = bounds[blockIdx.x]; bn = bounds[blockIdx.x + 1]; }
  for (int64_t tk = blockIdx.x; tk < ntile; tk += gridDim.x) {   // block-uniform
    const int64_t a = an, b = bn;
    if (tk + gridDim.x < ntile) { an = bounds[tk + gridDim.x]; bn = bounds[tk + gridDim.x + 1]; }
    if (a < 0 || b < 0) continue;   // flagged: the host redoes the sort
    const int m = (int)(b - a);     // <= LSTEP + RUN_MAX = LCAP
    // the tile's rows: all LPT loads of a thread issued together; a row's input index stays in a
    // register for the write-out (thread t handles rows t + k LT in both phases)
    uint4 v[LPT];
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = t + k * LT;
      if (i < m) v[k] = rec_in[a + i];
    }
    uint32_t row[LPT];
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = t + k * LT;
      row[k] = v[k].z;
      if (i < m) {
        const uint64_t zz = rec_z(v[k]);
        s_z[i] = zz; s_bs[i] = v[k].w; s_run[i] = prefix4(v[k].w, zz, po, pw);
      }
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
#pragma unroll
    for (int k = 0; k < LPT; ++k) {
      const int i = t + k * LT;
      if (i >= m) continue;
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
      bin_out[dst] = SH ? bs_bin(bi, sq, binhi) : (uint16_t)bi;
      if (SH) sh_out[dst] = (uint8_t)(bi >> sq);
      perm_out[dst] = (int64_t)row[k];
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(STPB) void k_widen_perm(int64_t n, int64_t* __restrict__ p64) {
  for (int64_t i = (int64_t)blockIdx.x * STPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * STPB) p64[i] = i;
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
    if (sh) o[k++] = sh[i];
    if (bin) {   // no bin: the Z2 / XZ2 layout [shard][z BE64]
      const uint16_t b = (uint16_t)bin[i];
      o[k++] = (uint8_t)(b >> 8);
      o[k++] = (uint8_t)b;
    }
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

// The digits of one sort, from the OR / AND of the keys: `lsd` = every byte on which some keys differ
// (LSD order); prefix mode = npre digits of pw <= 9 bits, each ending at the highest varying bit below
// the previous one (only constant bits are skipped), over the top ~log2(n) - 1 varying bits (runs of
// ~2 equal prefixes for uniform keys), when that is fewer passes than the varying bytes
struct SortPlan {
  std::vector<int> lsd;
  int npre = 0, pw = 0, pofs[4] = {-1, -1, -1, -1};
  bool prefix = false;
  int sq = 16;            // the shard's bit in bs (squeeze_bs), and bin's constant bits above it
  uint32_t binhi = 0;
  std::vector<int> first_offs() const {   // the first digit passes, LSD order
    if (!prefix) return lsd;
    std::vector<int> o(pofs, pofs + npre);
    std::reverse(o.begin(), o.end());
    return o;
  }
  DigitOffs first_digits() const {
    DigitOffs o{};
    const std::vector<int> f = first_offs();
    o.np = (int)f.size();
    for (int k = 0; k < o.np; ++k) { o.off[k] = f[k]; o.w[k] = prefix ? pw : 8; }
    return o;
  }
};
inline bool operator==(const DigitOffs& a, const DigitOffs& b) {
  if (a.np != b.np) return false;
  for (int k = 0; k < a.np; ++k)
    if (a.off[k] != b.off[k] || a.w[k] != b.w[k]) return false;
  return true;
}
static SortPlan plan_sort(const unsigned long long h_raw[4], bool sh, int64_t n, int sort_mode) {
  SortPlan p;
  unsigned long long h[4] = {h_raw[0], h_raw[1], h_raw[2], h_raw[3]};
  if (sh) {   // the digits are planned over the squeezed key (squeeze_bs)
    const uint32_t vbin = (uint32_t)((h_raw[1] ^ h_raw[3]) & 0xffffu);
    p.sq = vbin ? 32 - __builtin_clz(vbin) : 0;
    p.binhi = (uint32_t)h_raw[3] & 0xffffu & ~((1u << p.sq) - 1u);
    auto sqz = [&](unsigned long long b) {
      return (unsigned long long)(((uint32_t)b & ((1u << p.sq) - 1u)) | (((uint32_t)b >> 16) << p.sq));
    };
    h[1] = sqz(h_raw[1]);
    h[3] = sqz(h_raw[3]);
  }
  for (int b = 0; b < NPASS; ++b) {
    if (b == 10 && !sh) continue;
    const uint64_t o = b < 8 ? h[0] >> (8 * b) : h[1] >> (8 * (b - 8));
    const uint64_t a = b < 8 ? h[2] >> (8 * b) : h[3] >> (8 * (b - 8));
    if (((o ^ a) & 255u) != 0) p.lsd.push_back(8 * b);
  }
  if (p.lsd.empty()) return p;
  const uint64_t vz = h[0] ^ h[2], vb = (h[1] ^ h[3]) & 0xffffffull;
  auto varying = [&](int bit) -> bool { return bit < 64 ? ((vz >> bit) & 1u) : ((vb >> (bit - 64)) & 1u); };
  int lg = 0;
  while (((int64_t)1 << lg) < n) ++lg;
  const int pbits = std::max(1, lg - 1);
  p.npre = std::min(4, (pbits + WMAX - 1) / WMAX);
  p.pw = std::min(WMAX, (pbits + p.npre - 1) / p.npre);
  int nfound = 0;
  int bit = 87;
  for (int k = 0; k < p.npre; ++k) {
    while (bit >= 0 && !varying(bit)) --bit;
    if (bit < 0) break;
    p.pofs[k] = std::max(0, bit - (p.pw - 1));
    bit = p.pofs[k] - 1;
    ++nfound;
  }
  p.prefix = sort_mode == 0 && (int)p.lsd.size() > p.npre && nfound == p.npre;
  return p;
}

// ------------------------------------------------------------------ key-range partition (multi-GPU ingest)
// A table split into `nd` contiguous key ranges (tablets / regions; one per GPU) by nd - 1 ascending
// splitter keys: row r goes to destination d = the number of splitters <= its key (a key equal to a
// splitter opens the upper range).  Keys compare as the row bytes do: (shard << 16 | bin as u16, z as
// u64), unsigned.  One read counts every tile's rows per destination (k_part_count), a device scan of
// those counts in destination-major order gives each (destination, tile) its output start, and a
// second read (k_part_scatter) ranks the tile's rows per destination in LDS (wave ballots, stable:
// within a destination rows keep their input order) and writes them as contiguous destination runs,
// so that destination d's rows are one slice of every output column -- what one all-to-all sends.
constexpr int XT = 256;                  // partition threads per block
constexpr int XTILE = 2048;              // rows per tile: wave w owns rows [512 w, 512 w + 512)
constexpr int XSLOT = XTILE / XT;        // 8 rows per lane, one per 64-row slot
constexpr int XMAX = 256;                // destinations at most (ranks of the partitioned table)

struct SplitLds {
  uint32_t hi[XMAX];
  uint64_t lo[XMAX];
};
// destination of key (hi, lo): first splitter greater than the key (binary search, ns < XMAX)
__device__ __forceinline__ int part_dest(const SplitLds& s, int ns, uint32_t hi, uint64_t lo) {
  int a = 0, b = ns;
  while (a < b) {
    const int m = (a + b) >> 1;
    const bool le = s.hi[m] < hi || (s.hi[m] == hi && s.lo[m] <= lo);
    if (le) a = m + 1;
    else b = m;
  }
  return a;
}
__device__ __forceinline__ void load_splitters(SplitLds& s, const uint64_t* __restrict__ split, int ns) {
  for (int k = threadIdx.x; k < ns; k += blockDim.x) {
    s.hi[k] = (uint32_t)split[2 * k];
    s.lo[k] = split[2 * k + 1];
  }
}
// lanes of this wave whose destination equals mine (among the lanes with `ok`), from nbits ballots
__device__ __forceinline__ uint64_t match_dest(uint32_t d, bool ok, int nbits) {
  uint64_t m = __ballot(ok);
  for (int bit = 0; bit < nbits; ++bit) {   // uniform
    const uint64_t b = __ballot((d >> bit) & 1u);
    m &= ((d >> bit) & 1u) ? b : ~b;
  }
  return m;
}
template <bool SH>
__device__ __forceinline__ void part_load_tile(const KeyCols& c, int64_t t0, int64_t n, uint64_t (&z)[XSLOT],
                                               uint32_t (&bs)[XSLOT]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = t0 + wave * (64 * XSLOT) + lane;
  if (t0 + XTILE <= n) {   // uniform: a full tile's loads are unconditional, all in flight together
#pragma unroll
    for (int s = 0; s < XSLOT; ++s) {
      z[s] = c.z[r0 + 64 * s];
      bs[s] = (uint32_t)c.bin[r0 + 64 * s] | (SH ? (uint32_t)c.sh[r0 + 64 * s] << 16 : 0u);
    }
  } else {
#pragma unroll
    for (int s = 0; s < XSLOT; ++s) {
      const int64_t r = r0 + 64 * s;
      z[s] = r < n ? c.z[r] : 0ull;
      bs[s] = r < n ? ((uint32_t)c.bin[r] | (SH ? (uint32_t)c.sh[r] << 16 : 0u)) : 0u;
    }
  }
}

// cnt[d * ntiles + tile] = rows of the tile bound for d (destination-major: the exclusive scan of cnt
// is each (destination, tile)'s first output row; the destinations' totals come from that scan, not from
// per-block device atomics -- eight counters taking one atomic per block each serialised the count pass:
// 1.59 ms per 250M rows)
template <bool SH>
__global__ __launch_bounds__(XT) void k_part_count(KeyCols c, int64_t n, const uint64_t* __restrict__ split, int ns,
                                                   int nbits, uint32_t* __restrict__ cnt, int64_t ntiles) {
  __shared__ SplitLds s_sp;
  __shared__ uint32_t s_c[XMAX];
  const int nd = ns + 1, lane = threadIdx.x & 63;
  load_splitters(s_sp, split, ns);
  for (int d = threadIdx.x; d < nd; d += XT) s_c[d] = 0u;
  __syncthreads();
  const int64_t tile = blockIdx.x, t0 = tile * XTILE;
  uint64_t z[XSLOT];
  uint32_t bs[XSLOT];
  part_load_tile<SH>(c, t0, n, z, bs);
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < XSLOT; ++s) {
    const bool ok = t0 + wave * (64 * XSLOT) + 64 * s + lane < n;
    const uint32_t d = ok ? (uint32_t)part_dest(s_sp, ns, bs[s], z[s]) : 0u;
    const uint64_t m = match_dest(d, ok, nbits);
    if (ok && (m & lanemask_lt()) == 0) atomicAdd(&s_c[d], (uint32_t)__popcll(m));   // one add per destination
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nd; d += XT) cnt[(int64_t)d * ntiles + tile] = s_c[d];
}

// each destination's row count from the destination-major scan: start of d = offs[d * ntiles]
__global__ __launch_bounds__(XMAX) void k_part_totals(const int64_t* __restrict__ offs, int64_t ntiles, int nd,
                                                      const int64_t* __restrict__ total, int64_t* __restrict__ out) {
  const int d = threadIdx.x;
  if (d < nd) out[d] = (d + 1 < nd ? offs[(int64_t)(d + 1) * ntiles] : *total) - offs[(int64_t)d * ntiles];
}

// The tile ranked per destination in LDS and written as destination runs.  offs = the exclusive scan
// of k_part_count's cnt.  Per row: z_out, bin_out, shard_out (SH), and the row's source as ids_out =
// ids[row] (IDS) or id_base + row, and / or rows_out = row (u32); either output may be null.
template <bool SH, bool IDS>
__global__ __launch_bounds__(XT) void k_part_scatter(KeyCols c, int64_t n, const uint64_t* __restrict__ split, int ns,
                                                     int nbits, const int64_t* __restrict__ offs, int64_t ntiles,
                                                     const int64_t* __restrict__ ids, int64_t id_base,
                                                     int64_t* __restrict__ ids_out, uint32_t* __restrict__ rows_out,
                                                     uint8_t* __restrict__ sh_out, uint16_t* __restrict__ bin_out,
                                                     uint64_t* __restrict__ z_out) {
  __shared__ SplitLds s_sp;
  __shared__ uint4 s_rec[XTILE];                 // {z lo, z hi, bs, tile row | destination << 16}
  __shared__ uint16_t s_wcnt[XT / 64][XMAX];     // per wave: rows of each destination (then: wave offsets)
  __shared__ uint32_t s_dstart[XMAX];            // the destination's first slot in the tile
  __shared__ int64_t s_g[XMAX];                  // output row of tile slot q = s_g[d] + q
  __shared__ uint32_t s_wsum[XT / 64];
  const int nd = ns + 1, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  load_splitters(s_sp, split, ns);
  for (int i = t; i < (XT / 64) * XMAX; i += XT) (&s_wcnt[0][0])[i] = 0;
  __syncthreads();
  const int64_t tile = blockIdx.x, t0 = tile * XTILE;
  uint64_t z[XSLOT];
  uint32_t bs[XSLOT];
  part_load_tile<SH>(c, t0, n, z, bs);
  uint32_t rd[XSLOT];   // wave rank | destination << 16; rank 0xffff = no row
  const uint64_t lt = lanemask_lt();
#pragma unroll
  for (int s = 0; s < XSLOT; ++s) {
    const bool ok = t0 + wave * (64 * XSLOT) + 64 * s + lane < n;
    const uint32_t d = ok ? (uint32_t)part_dest(s_sp, ns, bs[s], z[s]) : 0u;
    const uint64_t m = match_dest(d, ok, nbits);
    const int r = __popcll(m & lt);
    const uint32_t c0 = s_wcnt[wave][d];
    rd[s] = (ok ? c0 + r : 0xffffu) | (d << 16);
    __builtin_amdgcn_wave_barrier();
    if (ok && r == 0) s_wcnt[wave][d] = (uint16_t)(c0 + __popcll(m));
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  // thread d: its wave offsets and tile total, then a block scan of the totals over destinations
  uint32_t tot = 0;
  if (t < nd) {
#pragma unroll
    for (int v = 0; v < XT / 64; ++v) {
      const uint32_t cv = s_wcnt[v][t];
      s_wcnt[v][t] = (uint16_t)tot;
      tot += cv;
    }
  }
  uint32_t x = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wsum[wave] = x;
  __syncthreads();
  if (t < nd) {
    uint32_t p = 0;
    for (int v = 0; v < wave; ++v) p += s_wsum[v];
    const uint32_t ds = p + x - tot;
    s_dstart[t] = ds;
    s_g[t] = offs[(int64_t)t * ntiles + tile] - (int64_t)ds;
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < XSLOT; ++s) {
    const uint32_t r = rd[s] & 0xffffu, d = rd[s] >> 16;
    if (r == 0xffffu) continue;
    const uint32_t row = (uint32_t)(wave * (64 * XSLOT) + 64 * s + lane);
    s_rec[s_dstart[d] + s_wcnt[wave][d] + r] = make_uint4((uint32_t)z[s], (uint32_t)(z[s] >> 32), bs[s], row | (d << 16));
  }
  __syncthreads();
  const int cntt = (int)min((int64_t)XTILE, n - t0);
  for (int q = t; q < cntt; q += XT) {
    const uint4 v = s_rec[q];
    const int64_t g = s_g[v.w >> 16] + q;
    const int64_t row = t0 + (v.w & 0xffffu);
    z_out[g] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    bin_out[g] = (uint16_t)v.z;
    if (SH) sh_out[g] = (uint8_t)(v.z >> 16);
    if (ids_out) ids_out[g] = IDS ? ids[row] : id_base + row;
    if (rows_out) rows_out[g] = (uint32_t)row;
  }
}

// n_samples keys at rows floor((2i + 1) n / (2 n_samples)): out[2i] = shard << 16 | bin (u16), out[2i + 1] = z
template <bool SH>
__global__ __launch_bounds__(256) void k_key_sample(KeyCols c, int64_t n, int ns, uint64_t* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= ns) return;
  const int64_t r = (int64_t)((uint64_t)(2 * i + 1) * (uint64_t)n / (2 * (uint64_t)ns));   // < 2^49: ns <= 2^16, n < 2^32
  out[2 * i] = (uint64_t)c.bin[r] | (SH ? (uint64_t)c.sh[r] << 16 : 0ull);
  out[2 * i + 1] = c.z[r];
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

int gm_z2_key_bytes(gm_ctx* ctx, const uint8_t* shard, const int64_t* z, int64_t n, uint8_t* out) {
  if (!ctx || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!z || !out) return GM_E_INVALID;
  hipLaunchKernelGGL(k_key_bytes, dim3((unsigned)((n + STPB - 1) / STPB)), dim3(STPB), 0, ctx->stream, shard, nullptr, z,
                     n, shard ? 9 : 8, out);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

int gm_sort_keys(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                 uint8_t* shard_out, int16_t* bin_out, int64_t* z_out, int64_t* perm_out) {
  if (!ctx || n < 0 || n > (int64_t)UINT32_MAX) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!z || !z_out || !perm_out || ((shard == nullptr) != (shard_out == nullptr)) ||
      ((bin == nullptr) != (bin_out == nullptr)))
    return GM_E_INVALID;
  hipStream_t s = ctx->stream;
  if (!bin) {
    // no time bin (Z2 / XZ2 tables): the sort runs over a zero bin column (constant, so no digit pass
    // looks at it) and its bin output goes to scratch
    void* zb = nullptr;
    int rc = ctx_workspace(ctx, WS_SCAN, (((size_t)n * 2 + 15) & ~(size_t)15) * 2, &zb);
    if (rc) return rc;
    bin = (const int16_t*)zb;
    bin_out = (int16_t*)((char*)zb + (((size_t)n * 2 + 15) & ~(size_t)15));
    GM_HIP(hipMemsetAsync(zb, 0, (size_t)n * 2, s));
  }
  const uint8_t* sh = shard;
  const KeyCols in{sh, (const uint16_t*)bin, (const uint64_t*)z};
  // 16-B z / 4-B bin / 2-B shard pair loads need aligned caller columns
  const int user_vec = ((uintptr_t)z % 16) == 0 && ((uintptr_t)bin % 4) == 0 && (!sh || ((uintptr_t)sh % 2) == 0);
  // 16-B loads of every column in the OR/AND and count reads
  const int user_wide = ((uintptr_t)z % 16) == 0 && ((uintptr_t)bin % 16) == 0 && (!sh || ((uintptr_t)sh % 16) == 0);
  const int64_t nchunk = (n + RCH - 1) / RCH;
#ifndef GM_SORT_CGRID   // count blocks: 1024 vs 512 -0.04 ms per sort, 256 +0.07 (profiles/r5/sort_count_grid_ab.txt)
#define GM_SORT_CGRID 1024
#endif
  const int cgrid = (int)std::max<int64_t>(1, std::min<int64_t>(GM_SORT_CGRID, (nchunk + CT / 64 - 1) / (CT / 64)));
  const int64_t ntiles = (n + PTILE - 1) / PTILE;
  uint4 *rec[2] = {nullptr, nullptr};
  unsigned long long* status = nullptr;
  uint32_t* counts = nullptr;
  unsigned int* ctr = nullptr;
  int64_t* lbounds = nullptr;
  size_t counts_bytes = 0;
  {  // context-owned workspace: records x 2 | granules | counts | tile counters | local bounds, 16-B aligned
    auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
    const size_t a_r = al((size_t)n * 16), a_st = al((size_t)ntiles * NB_MAX * 8), a_c = al((size_t)MAXTAG * NB_MAX * 4),
                 a_t = al((size_t)MAXTAG * 4), a_b = al((size_t)((n + LSTEP - 1) / LSTEP + 1) * 8);
    void* base = nullptr;
    int wrc = ctx_workspace(ctx, WS_SORT, 2 * a_r + a_st + a_c + a_t + a_b, &base);
    if (wrc) return wrc;
    char* q = (char*)base;
    rec[0] = (uint4*)q; q += a_r;
    rec[1] = (uint4*)q; q += a_r;
    status = (unsigned long long*)q; q += a_st;
    counts = (uint32_t*)q; q += a_c;
    ctr = (unsigned int*)q; q += a_t;
    lbounds = (int64_t*)q;
    counts_bytes = a_c;
    GM_HIP(hipMemsetAsync(status, 0, a_st + a_c + a_t, s));   // granules (tag 0 = none), counts, counters
  }
  // which key bits vary: acc[0..3] = OR z, OR bs, AND z, AND bs of every key (k_sort_count), acc[8..11]
  // the same over a sample (k_key_or_and_sample), acc[4] k_sort_local's flag
  unsigned long long* acc = (unsigned long long*)ctx->d_scratch;
  GM_HIP(hipMemsetAsync(acc, 0, 16, s));
  GM_HIP(hipMemsetAsync(acc + 2, 0xff, 16, s));
  GM_HIP(hipMemsetAsync(acc + 4, 0, 8, s));
  GM_HIP(hipMemsetAsync(acc + 8, 0, 16, s));
  GM_HIP(hipMemsetAsync(acc + 10, 0xff, 16, s));
  if (sh) hipLaunchKernelGGL(k_key_or_and_sample<true>, dim3(SAMPLE / 256), dim3(256), 0, s, in, n, acc + 8);
  else hipLaunchKernelGGL(k_key_or_and_sample<false>, dim3(SAMPLE / 256), dim3(256), 0, s, in, n, acc + 8);
  GM_CHECK_LAUNCH();
  unsigned long long hs[4];
  GM_HIP(hipMemcpyAsync(hs, acc + 8, sizeof(hs), hipMemcpyDeviceToHost, s));
  GM_HIP(hipStreamSynchronize(s));
  const SortPlan guess = plan_sort(hs, sh != nullptr, n, ctx->sort_mode);
  // the guessed plan's first digit set counted in the read that takes the exact OR / AND
  {
    const DigitOffs o = guess.first_digits();
    if (sh) hipLaunchKernelGGL((k_sort_count<true, true>), dim3(cgrid), dim3(CT), 0, s, in, n, o, counts, user_wide, acc, guess.sq);
    else hipLaunchKernelGGL((k_sort_count<false, true>), dim3(cgrid), dim3(CT), 0, s, in, n, o, counts, user_wide, acc, 16);
    GM_CHECK_LAUNCH();
  }
  unsigned long long hacc[4];
  GM_HIP(hipMemcpyAsync(hacc, acc, sizeof(hacc), hipMemcpyDeviceToHost, s));
  GM_HIP(hipStreamSynchronize(s));
  const SortPlan plan = plan_sort(hacc, sh != nullptr, n, ctx->sort_mode);
  const std::vector<int>& lsd = plan.lsd;
  if (lsd.empty()) {  // every key equal: table order = input order
    if (sh) GM_HIP(hipMemcpyAsync(shard_out, sh, (size_t)n, hipMemcpyDeviceToDevice, s));
    GM_HIP(hipMemcpyAsync(bin_out, bin, (size_t)n * 2, hipMemcpyDeviceToDevice, s));
    GM_HIP(hipMemcpyAsync(z_out, z, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_widen_perm, dim3((unsigned)std::min<int64_t>(4096, (n + STPB - 1) / STPB)), dim3(STPB), 0, s, n,
                       perm_out);
    GM_CHECK_LAUNCH();
    ctx->sort_last = 0;
    return GM_OK;
  }
  // the sample's plan holds when the exact bits give the same first digits; else count again
  bool counted = guess.first_digits() == plan.first_digits() && guess.sq == plan.sq;
  if (!counted) GM_HIP(hipMemsetAsync(counts, 0, counts_bytes, s));
  const bool prefix_mode = plan.prefix;
  const int npre = plan.npre, pw = plan.pw;
  const int* pofs = plan.pofs;
  // digit passes at bit offsets `offs` (LSD order) from the caller's columns, tags tag0 + 1...; the
  // last pass lands in the user outputs when `to_user_last`, else in records (*last_rec)
  const uint4* last_rec = nullptr;
  auto passes = [&](const std::vector<int>& offs, int w, bool to_user_last, int tag0) -> int {
    const int np = (int)offs.size();
    DigitOffs o{};
    o.np = np;
    for (int k = 0; k < np; ++k) { o.off[k] = offs[k]; o.w[k] = w; }
    uint32_t* cnt = counts + (size_t)tag0 * NB_MAX;
    if (!counted) {
      if (sh) hipLaunchKernelGGL((k_sort_count<true, false>), dim3(cgrid), dim3(CT), 0, s, in, n, o, cnt, user_wide, nullptr, plan.sq);
      else hipLaunchKernelGGL((k_sort_count<false, false>), dim3(cgrid), dim3(CT), 0, s, in, n, o, cnt, user_wide, nullptr, 16);
      if (hipGetLastError() != hipSuccess) return hip_fail(hipErrorLaunchFailure, "k_sort_count");
    }
    counted = false;   // a later call (the fallback) counts its own digits
    for (int k = 0; k < np; ++k) {
      PassArgs a{};
      a.in = in;
      a.rec_in = k > 0 ? rec[(k - 1) & 1] : nullptr;
      a.sh_out = shard_out; a.bin_out = (uint16_t*)bin_out; a.z_out = (uint64_t*)z_out; a.perm_out = perm_out;
      a.rec_out = rec[k & 1];
      a.n = n; a.off = offs[k]; a.w = w; a.tag = (uint32_t)(tag0 + k + 1);
      a.counts = cnt + (size_t)k * NB_MAX;
      a.status = status;
      a.ctr = ctr + tag0 + k;
      a.vec = user_vec;
      a.sq = plan.sq; a.binhi = plan.binhi;
      const bool first = k == 0, user = to_user_last && k == np - 1;
      void (*kern)(PassArgs) =
          sh ? (first ? (user ? k_sort_pass<false, true, true> : k_sort_pass<false, false, true>)
                      : (user ? k_sort_pass<true, true, true> : k_sort_pass<true, false, true>))
             : (first ? (user ? k_sort_pass<false, true, false> : k_sort_pass<false, false, false>)
                      : (user ? k_sort_pass<true, true, false> : k_sort_pass<true, false, false>));
      hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(PT), 0, s, a);
      if (hipGetLastError() != hipSuccess) return hip_fail(hipErrorLaunchFailure, "k_sort_pass");
      last_rec = rec[k & 1];
    }
    return GM_OK;
  };
  if (prefix_mode) {
    int rc = passes(plan.first_offs(), pw, false, 0);
    if (rc) return rc;
    const int4 po = make_int4(pofs[0], pofs[1], pofs[2], pofs[3]);
    const int lgrid = resident_blocks((const void*)k_sort_local<false>, ctx->device, LT, 2);
    const int64_t nbound = (n + LSTEP - 1) / LSTEP + 1;
    hipLaunchKernelGGL(k_local_bounds, dim3((unsigned)((nbound + 3) / 4)), dim3(256), 0, s, last_rec, n, po, pw, lbounds,
                       (uint32_t*)(acc + 4));
    if (sh)
      hipLaunchKernelGGL(k_sort_local<true>, dim3(lgrid), dim3(LT), 0, s, last_rec, shard_out, (uint16_t*)bin_out,
                         (uint64_t*)z_out, perm_out, n, po, pw, (uint32_t*)(acc + 4), lbounds, plan.sq, plan.binhi);
    else
      hipLaunchKernelGGL(k_sort_local<false>, dim3(lgrid), dim3(LT), 0, s, last_rec, nullptr, (uint16_t*)bin_out,
                         (uint64_t*)z_out, perm_out, n, po, pw, (uint32_t*)(acc + 4), lbounds, plan.sq, plan.binhi);
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
  return passes(lsd, 8, true, prefix_mode ? npre : 0);
}

int gm_key_sample(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n, int32_t n_samples,
                  uint64_t* key_hi, uint64_t* key_lo) {
  if (!ctx || n < 0 || n > (int64_t)UINT32_MAX || n_samples < 0 || n_samples > 65536) return GM_E_INVALID;
  if (n == 0 || n_samples == 0) return GM_OK;
  if (!bin || !z || !key_hi || !key_lo) return GM_E_INVALID;
  void* ws = nullptr;
  int rc = ctx_workspace(ctx, WS_SCAN, (size_t)n_samples * 16, &ws);
  if (rc) return rc;
  const KeyCols in{shard, (const uint16_t*)bin, (const uint64_t*)z};
  const dim3 g((unsigned)((n_samples + 255) / 256));
  if (shard) hipLaunchKernelGGL(k_key_sample<true>, g, dim3(256), 0, ctx->stream, in, n, (int)n_samples, (uint64_t*)ws);
  else hipLaunchKernelGGL(k_key_sample<false>, g, dim3(256), 0, ctx->stream, in, n, (int)n_samples, (uint64_t*)ws);
  GM_CHECK_LAUNCH();
  std::vector<uint64_t> h((size_t)n_samples * 2);
  rc = copy_d2h(ctx, h.data(), ws, h.size() * 8);
  if (rc) return rc;
  for (int32_t i = 0; i < n_samples; ++i) {
    key_hi[i] = h[2 * (size_t)i];
    key_lo[i] = h[2 * (size_t)i + 1];
  }
  return GM_OK;
}

int gm_key_partition(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                     const uint64_t* split_hi, const uint64_t* split_lo, int32_t n_split, const int64_t* ids,
                     int64_t id_base, uint8_t* shard_out, int16_t* bin_out, int64_t* z_out, int64_t* ids_out,
                     uint32_t* rows_out, int64_t* dest_counts) {
  if (!ctx || n < 0 || n > (int64_t)UINT32_MAX || n_split < 0 || n_split >= XMAX || !dest_counts) return GM_E_INVALID;
  if (n_split > 0 && (!split_hi || !split_lo)) return GM_E_INVALID;
  for (int32_t k = 0; k < n_split; ++k) {   // ascending splitters, keys of 24 bits + 64 bits
    if (split_hi[k] >> 24) return set_error("gm_key_partition: splitter hi past 24 bits"), GM_E_INVALID;
    if (k > 0 && (split_hi[k] < split_hi[k - 1] || (split_hi[k] == split_hi[k - 1] && split_lo[k] < split_lo[k - 1])))
      return set_error("gm_key_partition: splitters not ascending"), GM_E_INVALID;
  }
  const int nd = n_split + 1;
  for (int d = 0; d < nd; ++d) dest_counts[d] = 0;
  if (n == 0) return GM_OK;
  if (!bin || !z || !bin_out || !z_out || ((shard == nullptr) != (shard_out == nullptr))) return GM_E_INVALID;
  hipStream_t s = ctx->stream;
  const int64_t ntiles = (n + XTILE - 1) / XTILE, ncnt = ntiles * nd;
  // workspace: splitters | counts (u32, destination-major) | their scan (i64) | scan partials | totals
  auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
  const size_t a_s = al((size_t)std::max(1, n_split) * 16), a_c = al((size_t)ncnt * 4), a_o = al((size_t)ncnt * 8),
               a_p = al((size_t)scan_partials_len(ncnt) * 8), a_t = al((size_t)(nd + 1) * 8);
  void* base = nullptr;
  int rc = ctx_workspace(ctx, WS_SCAN, a_s + a_c + a_o + a_p + a_t, &base);
  if (rc) return rc;
  char* q = (char*)base;
  uint64_t* split = (uint64_t*)q; q += a_s;
  uint32_t* cnt = (uint32_t*)q; q += a_c;
  int64_t* offs = (int64_t*)q; q += a_o;
  int64_t* partials = (int64_t*)q; q += a_p;
  int64_t* dtot = (int64_t*)q;   // [nd] destination totals, then the scan's grand total
  if (n_split > 0) {
    std::vector<uint64_t> hs((size_t)n_split * 2);
    for (int32_t k = 0; k < n_split; ++k) { hs[2 * (size_t)k] = split_hi[k]; hs[2 * (size_t)k + 1] = split_lo[k]; }
    rc = copy_h2d(ctx, split, hs.data(), hs.size() * 8);
    if (rc) return rc;
  }
  int nbits = 0;
  while ((1 << nbits) < nd) ++nbits;
  const KeyCols in{shard, (const uint16_t*)bin, (const uint64_t*)z};
  const dim3 grid((unsigned)ntiles);
  if (shard) hipLaunchKernelGGL(k_part_count<true>, grid, dim3(XT), 0, s, in, n, split, n_split, nbits, cnt, ntiles);
  else hipLaunchKernelGGL(k_part_count<false>, grid, dim3(XT), 0, s, in, n, split, n_split, nbits, cnt, ntiles);
  GM_CHECK_LAUNCH();
  launch_excl_scan<uint32_t, int64_t>(s, cnt, ncnt, offs, partials, dtot + nd);
  hipLaunchKernelGGL(k_part_totals, dim3(1), dim3(XMAX), 0, s, offs, ntiles, nd, dtot + nd, dtot);
  GM_CHECK_LAUNCH();
  void (*kern)(KeyCols, int64_t, const uint64_t*, int, int, const int64_t*, int64_t, const int64_t*, int64_t, int64_t*,
               uint32_t*, uint8_t*, uint16_t*, uint64_t*) =
      shard ? (ids ? k_part_scatter<true, true> : k_part_scatter<true, false>)
            : (ids ? k_part_scatter<false, true> : k_part_scatter<false, false>);
  hipLaunchKernelGGL(kern, grid, dim3(XT), 0, s, in, n, split, n_split, nbits, offs, ntiles, ids, id_base, ids_out, rows_out,
                     shard_out, (uint16_t*)bin_out, (uint64_t*)z_out);
  GM_CHECK_LAUNCH();
  return copy_d2h(ctx, dest_counts, dtot, (size_t)nd * 8);
}

}  // extern "C"
