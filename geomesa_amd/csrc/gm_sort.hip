// gm_sort.hip -- the sorted key table: row-key bytes, device sort into table order, and range scans.
//
// A GeoMesa Z3 table is the set of row keys [shard?][bin BE16][z BE64][id] kept in byte order by the
// store (Z3IndexKeySpace.toIndexKey, idx/index/z3/Z3IndexKeySpace.scala:63-95; ByteArrays.writeShort /
// writeLong, geomesa-utils/.../index/ByteArrays.scala:51,90-99).  A query seeks each byte range
// getRangeBytes produces (Z3IndexKeySpace.scala:196-238) and the tablet server runs the Z3Filter on
// every row inside (RowFilterIterator.scala:52-66).  Here the table is columnar and resident in HBM:
//   * gm_z3_key_bytes  -- the row-key prefix bytes, staged through LDS so the stores are 16-B wide;
//   * gm_sort_keys     -- a stable LSD radix sort of (shard u8, bin u16, z u64) in that byte order,
//                         8-bit digits, per-block segments: histogram -> one-block scan -> stable
//                         scatter (wave ballots rank equal digits, LDS reorders each 2048-row tile so
//                         the global writes are digit runs).  Passes on which every key has the same
//                         digit are skipped (one extra read computes all 11 digit histograms);
// The range scan over a sorted table (gm_key_range_scan) lives with the other row-filter scans in
// gm_filter.hip.
#include <string.h>

#include <algorithm>
#include <vector>

#include "gm_scan.hpp"

namespace gm {

constexpr int STPB = 256;               // sort / scan threads per block
constexpr int SPER = 8;                 // rows per thread per tile
constexpr int STILE = STPB * SPER;      // 2048 rows per tile
constexpr int SNW = STPB / 64;          // waves per block
constexpr int NPASS = 11;               // digit positions: z bytes 0..7, bin bytes 0..1, shard

__device__ __forceinline__ uint32_t key_digit(uint8_t sh, uint16_t b, uint64_t z, int pass) {
  if (pass < 8) return (uint32_t)(z >> (8 * pass)) & 255u;
  if (pass < 10) return (uint32_t)(b >> (8 * (pass - 8))) & 255u;
  return sh;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// all 11 digit histograms in one read: a pass whose histogram has one bucket holding every key is
// skipped (its scatter would be the identity)
__global__ __launch_bounds__(STPB) void k_sort_hist_all(const uint8_t* __restrict__ sh, const uint16_t* __restrict__ bin,
                                                        const uint64_t* __restrict__ z, int64_t n,
                                                        uint32_t* __restrict__ ghist) {
  __shared__ uint32_t h[NPASS * 256];
  for (int i = threadIdx.x; i < NPASS * 256; i += STPB) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * STPB + threadIdx.x; i < n; i += (int64_t)gridDim.x * STPB) {
    const uint64_t zz = z[i];
    const uint16_t b = bin[i];
    const uint8_t s = sh ? sh[i] : 0;
#pragma unroll
    for (int p = 0; p < NPASS; ++p) atomicAdd(&h[p * 256 + key_digit(s, b, zz, p)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NPASS * 256; i += STPB)
    if (h[i]) atomicAdd(&ghist[i], h[i]);
}

// per-block segment histogram of one digit, digit-major: hist[d * gridDim.x + block]
__global__ __launch_bounds__(STPB) void k_sort_hist(const uint8_t* __restrict__ sh, const uint16_t* __restrict__ bin,
                                                    const uint64_t* __restrict__ z, int64_t n, int64_t per_block,
                                                    int pass, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(n, b0 + per_block);
  for (int64_t i = b0 + threadIdx.x; i < b1; i += STPB) {
    const uint32_t d = pass < 8 ? (uint32_t)(z[i] >> (8 * pass)) & 255u
                                : pass < 10 ? (uint32_t)(bin[i] >> (8 * (pass - 8))) & 255u : (uint32_t)sh[i];
    atomicAdd(&h[d], 1u);
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter of one digit pass.  Each block walks its segment in tiles of 2048 rows laid out
// slot-major (row = tile + k*256 + thread), which is also the order ranks are assigned in:
// within a wave, lanes holding the same digit find each other with 8 ballots (one per digit bit);
// per (slot, wave) digit counts are turned into running offsets per digit; the tile is written to
// LDS in digit order and streamed out as digit runs at the block's cursor for each digit.
__global__ __launch_bounds__(STPB) void k_sort_scatter(const uint8_t* __restrict__ sh_in, const uint16_t* __restrict__ bin_in,
                                                       const uint64_t* __restrict__ z_in,
                                                       const uint32_t* __restrict__ perm_in, uint8_t* __restrict__ sh_out,
                                                       uint16_t* __restrict__ bin_out, uint64_t* __restrict__ z_out,
                                                       uint32_t* __restrict__ perm_out, int64_t n, int64_t per_block,
                                                       int pass, const uint32_t* __restrict__ off) {
  __shared__ uint64_t s_z[STILE];
  __shared__ uint32_t s_perm[STILE];
  __shared__ uint16_t s_bin[STILE];
  __shared__ uint8_t s_sh[STILE];
  __shared__ uint16_t s_cnt[SPER * SNW][256];
  __shared__ uint32_t s_gcur[256], s_tot[256], s_dstart[256], s_wsum[SNW];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  s_gcur[t] = off[(int64_t)t * gridDim.x + blockIdx.x];
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(n, b0 + per_block);
  const uint64_t lt = lanemask_lt();
  for (int64_t t0 = b0; t0 < b1; t0 += STILE) {
    {
      uint4* c4 = (uint4*)&s_cnt[0][0];
      for (int i = t; i < SPER * SNW * 256 * 2 / 16; i += STPB) c4[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    uint64_t zv[SPER];
    uint32_t pv[SPER], dg[SPER];
    uint16_t bv[SPER];
    uint8_t sv[SPER];
    int rk[SPER];
#pragma unroll
    for (int k = 0; k < SPER; ++k) {
      const int64_t i = t0 + k * STPB + t;
      const bool ok = i < b1;
      zv[k] = 0; bv[k] = 0; sv[k] = 0; pv[k] = 0; dg[k] = 0;
      if (ok) {
        zv[k] = z_in[i];
        bv[k] = bin_in[i];
        sv[k] = sh_in ? sh_in[i] : 0;
        pv[k] = perm_in ? perm_in[i] : (uint32_t)i;
        dg[k] = key_digit(sv[k], bv[k], zv[k], pass);
      }
      uint64_t m = __ballot(ok);
#pragma unroll
      for (int bit = 0; bit < 8; ++bit) {
        const uint64_t bb = __ballot(ok && ((dg[k] >> bit) & 1u));
        m &= ((dg[k] >> bit) & 1u) ? bb : ~bb;
      }
      const uint64_t below = m & lt;
      rk[k] = ok ? __popcll(below) : -1;
      if (ok && below == 0) s_cnt[k * SNW + wave][dg[k]] = (uint16_t)__popcll(m);
    }
    __syncthreads();
    {  // running offsets per digit over the (slot, wave) order
      uint32_t run = 0;
      for (int s = 0; s < SPER * SNW; ++s) {
        const uint32_t c = s_cnt[s][t];
        s_cnt[s][t] = (uint16_t)run;
        run += c;
      }
      s_tot[t] = run;
      // exclusive scan of the digit totals across the block
      uint32_t x = run;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) s_wsum[wave] = x;
      __syncthreads();
      uint32_t pre = 0;
      for (int w = 0; w < wave; ++w) pre += s_wsum[w];
      s_dstart[t] = pre + x - run;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SPER; ++k) {
      if (rk[k] < 0) continue;
      const uint32_t pos = s_dstart[dg[k]] + s_cnt[k * SNW + wave][dg[k]] + (uint32_t)rk[k];
      s_z[pos] = zv[k]; s_bin[pos] = bv[k]; s_sh[pos] = sv[k]; s_perm[pos] = pv[k];
    }
    __syncthreads();
    const int cnt = (int)min((int64_t)STILE, b1 - t0);
    for (int q = t; q < cnt; q += STPB) {
      const uint32_t d = key_digit(s_sh[q], s_bin[q], s_z[q], pass);
      const int64_t g = (int64_t)s_gcur[d] + (q - (int)s_dstart[d]);
      z_out[g] = s_z[q];
      bin_out[g] = s_bin[q];
      if (sh_out) sh_out[g] = s_sh[q];
      perm_out[g] = s_perm[q];
    }
    __syncthreads();
    s_gcur[t] += s_tot[t];
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
  // which digit passes carry information
  uint32_t* ghist = nullptr;
  GM_HIP(hipMallocAsync((void**)&ghist, NPASS * 256 * 4, s));
  GM_HIP(hipMemsetAsync(ghist, 0, NPASS * 256 * 4, s));
  hipLaunchKernelGGL(k_sort_hist_all, dim3((unsigned)std::min<int64_t>(2048, (n + STPB - 1) / STPB)), dim3(STPB), 0, s, sh,
                     (const uint16_t*)bin, (const uint64_t*)z, n, ghist);
  GM_CHECK_LAUNCH();
  std::vector<uint32_t> h(NPASS * 256);
  GM_HIP(hipMemcpyAsync(h.data(), ghist, NPASS * 256 * 4, hipMemcpyDeviceToHost, s));
  GM_HIP(hipStreamSynchronize(s));
  GM_HIP(hipFreeAsync(ghist, s));
  std::vector<int> passes;
  for (int p = 0; p < NPASS; ++p) {
    if (p == 10 && !sh) continue;
    if (*std::max_element(h.begin() + p * 256, h.begin() + (p + 1) * 256) != (uint32_t)n) passes.push_back(p);
  }
  const int np = (int)passes.size();
  if (np == 0) {  // every key equal: table order = input order
    if (sh) GM_HIP(hipMemcpyAsync(shard_out, sh, (size_t)n, hipMemcpyDeviceToDevice, s));
    GM_HIP(hipMemcpyAsync(bin_out, bin, (size_t)n * 2, hipMemcpyDeviceToDevice, s));
    GM_HIP(hipMemcpyAsync(z_out, z, (size_t)n * 8, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_widen_perm, dim3((unsigned)std::min<int64_t>(4096, (n + STPB - 1) / STPB)), dim3(STPB), 0, s,
                       nullptr, n, perm_out);
    GM_CHECK_LAUNCH();
    return GM_OK;
  }
  // one resident wave of blocks: the scatter's LDS (~47 KiB) allows 3 blocks per CU, and a grid of
  // 1024 blocks ran as 768 + a second round of 256
  static int resident = 0;
  if (!resident) {
    int b = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_sort_scatter, STPB, 0) != hipSuccess || b < 1) b = 2;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess) cus = prop.multiProcessorCount;
    resident = b * cus;
  }
  const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(resident, (n + STILE - 1) / STILE));
  const int64_t per = ((n + nblk - 1) / nblk + STILE - 1) / STILE * STILE;
  const int grid = (int)((n + per - 1) / per);
  // ping-pong: the user outputs and one temp set; the last pass lands in the user outputs
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
  const uint8_t* ish = sh;
  const uint16_t* ibin = (const uint16_t*)bin;
  const uint64_t* iz = (const uint64_t*)z;
  const uint32_t* iperm = nullptr;
  int rc = GM_OK;
  for (int k = 0; k < np && !rc; ++k) {
    const bool to_user = ((np - 1 - k) % 2) == 0;
    uint8_t* osh = sh ? (to_user ? shard_out : tsh) : nullptr;
    uint16_t* obin = to_user ? (uint16_t*)bin_out : tbin;
    uint64_t* oz = to_user ? (uint64_t*)z_out : tz;
    uint32_t* operm = (k % 2) ? p1 : p0;
    hipLaunchKernelGGL(k_sort_hist, dim3(grid), dim3(STPB), 0, s, ish, ibin, iz, n, per, passes[k], hist);
    launch_excl_scan(s, hist, (int64_t)256 * grid, hist, hpart, (int64_t*)nullptr);
    hipLaunchKernelGGL(k_sort_scatter, dim3(grid), dim3(STPB), 0, s, ish, ibin, iz, iperm, osh, obin, oz, operm, n, per,
                       passes[k], hist);
    if (hipGetLastError() != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "k_sort_scatter");
    ish = osh; ibin = obin; iz = oz; iperm = operm;
  }
  if (!rc) {
    hipLaunchKernelGGL(k_widen_perm, dim3((unsigned)std::min<int64_t>(4096, (n + STPB - 1) / STPB)), dim3(STPB), 0, s,
                       iperm, n, perm_out);
    if (hipGetLastError() != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "k_widen_perm");
  }
  return rc;
}

}  // extern "C"
