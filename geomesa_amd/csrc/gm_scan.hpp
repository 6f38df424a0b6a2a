// gm_scan.hpp -- shared pieces of the mask -> block scan -> ordered compaction pipeline
// (gm_filter.hip; the fused query scan in gm_pip.hip).
#pragma once

#include "gm_internal.hpp"

namespace gm {

constexpr int FTPB = 256;             // threads per block
#ifndef GM_FELEMS
#define GM_FELEMS 16  // sweep (tools/filter_ab.sh, z3filter_scan ms per 1B rows): 4 2.27, 8 1.81-1.94, 16 1.68-1.80, 32 1.92-1.94
#endif
constexpr int FELEMS = GM_FELEMS;     // rows per thread per block
static_assert(FELEMS % 2 == 0 && FELEMS >= 2, "pair layout");
constexpr int FROWS = FTPB * FELEMS;  // rows per block (4096) -> 64 mask words

// ------------------------------------------------------------------ vectorised pass A
// The scalar kernels of gm_filter.hip move 2 B (bin) and 8 B (z) per lane per load instruction; on gfx950 narrow
// per-lane accesses stream at roughly half the 16-B rate.  The _v variants use the layout of the
// encode kernels: each lane takes PAIRS of consecutive rows, one 16-B load per 8-byte column
// (z, x, y, t) and one 4-B load of the two bins, and pair p of lane l in step u sits at
// block_base + u*256 + l, so every wave instruction reads one contiguous 1 KiB run.  A wave step
// covers 128 rows: ballot(row 2l) and ballot(row 2l+1) interleave bit by bit into the two 64-bit
// mask words of those rows.  A block still covers FROWS = 4096 rows (8 steps), so block_counts,
// the count scan and k_mask_to_ids are shared with the scalar kernels.
typedef short sv2 __attribute__((ext_vector_type(2)));
constexpr int FPAIRS = FELEMS / 2;   // pair steps per lane

// 32 -> 64-bit bit spread (bit k -> bit 2k)
__device__ __forceinline__ uint64_t spread2_32(uint32_t v) {
  return (uint64_t)spread2_16(v & 0xffffu) | ((uint64_t)spread2_16(v >> 16) << 32);
}

// the wave's two mask words from the even-row and odd-row ballots; lanes 0 and 1 store one each
__device__ __forceinline__ void put_pair_words(uint64_t even, uint64_t odd, uint64_t* __restrict__ mask, int64_t word,
                                               int64_t nwords) {
  const int lane = threadIdx.x & 63;
  if (lane < 2) {
    const uint32_t e = (uint32_t)(lane ? (even >> 32) : even), o = (uint32_t)(lane ? (odd >> 32) : odd);
    if (word + lane < nwords) mask[word + lane] = spread2_32(e) | (spread2_32(o) << 1);
  }
}

template <int TPB = FTPB>
__device__ __forceinline__ void block_count_waves(int wave_cnt, int32_t* block_counts) {
  __shared__ int s_wc[TPB / 64];
  if ((threadIdx.x & 63) == 0) s_wc[threadIdx.x >> 6] = wave_cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < TPB / 64; ++i) s += s_wc[i];
    block_counts[blockIdx.x] = s;
  }
}

// Row predicate over a pair layout: LOAD(p, u) stages pair p, ROW(u, j) evaluates row j (0/1) of the
// staged pair, TAIL(u) evaluates the odd last row n-1 (pair index n/2) with scalar loads.
template <class Load, class Row, class Tail>
__device__ __forceinline__ void pair_scan(int64_t n, uint64_t* __restrict__ mask, int32_t* __restrict__ block_counts,
                                          Load load, Row row, Tail tail) {
  const int64_t npairs = n >> 1, nwords = (n + 63) >> 6;
  const int wave = threadIdx.x >> 6;
  const int64_t pbase = (int64_t)blockIdx.x * (FTPB * FPAIRS);
#pragma unroll
  for (int u = 0; u < FPAIRS; ++u) {
    const int64_t p = pbase + (int64_t)u * FTPB + threadIdx.x;
    if (p < npairs) load(p, u);
  }
  int cnt = 0;
#pragma unroll
  for (int u = 0; u < FPAIRS; ++u) {
    const int64_t p = pbase + (int64_t)u * FTPB + threadIdx.x;
    bool e = false, o = false;
    if (p < npairs) { e = row(u, 0); o = row(u, 1); }
    else if (p == npairs && (n & 1)) e = tail(p);
    const uint64_t be = __ballot(e), bo = __ballot(o);
    cnt += __popcll(be) + __popcll(bo);
    put_pair_words(be, bo, mask, ((pbase + (int64_t)u * FTPB + wave * 64) * 2) >> 6, nwords);
  }
  block_count_waves(cnt, block_counts);
}

// Device-wide exclusive scan, two levels (block counts of the mask scans, radix-sort histograms).
// A single workgroup walking ~500k counts took 1.2-1.5 ms per call -- a third of the 1B-row scan
// it followed.
//   k_scan_partials: one block per SCAN_CHUNK values -> chunk sums
//   k_scan_chunks  : one workgroup scans the chunk sums (a few hundred) in place; total -> *total_out
//   k_scan_apply   : per chunk, block-wide exclusive scan + the chunk's base -> out[] (in place is fine:
//                    every thread reads its 16 values before writing them)
constexpr int SCAN_TPB = 256;
constexpr int SCAN_PER = 16;                          // consecutive counts per thread
constexpr int SCAN_CHUNK = SCAN_TPB * SCAN_PER;       // 4096 counts per block

// block-wide exclusive scan of one value per thread (256 threads); *total gets the block sum
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* total) {
  __shared__ int64_t s_w[SCAN_TPB / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t o = __shfl_up(inc, off, 64);
    if (lane >= off) inc += o;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  int64_t wbase = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < SCAN_TPB / 64; ++i) {
    if (i < w) wbase += s_w[i];
    tot += s_w[i];
  }
  *total = tot;
  return wbase + inc - v;
}

template <class TIn>
__global__ __launch_bounds__(SCAN_TPB) void k_scan_partials(const TIn* __restrict__ counts, int64_t nb,
                                                            int64_t* __restrict__ partials) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_CHUNK;
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    const int64_t j = base + (int64_t)i * SCAN_TPB + threadIdx.x;   // coalesced
    if (j < nb) s += counts[j];
  }
  int64_t tot;
  block_excl_scan(s, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

static __global__ __launch_bounds__(SCAN_TPB) void k_scan_chunks(int64_t* __restrict__ partials, int64_t np,
                                                          int64_t* __restrict__ total_out) {
  int64_t run = 0;
  for (int64_t c0 = 0; c0 < np; c0 += SCAN_TPB) {   // np is small: a few rounds at most
    const int64_t j = c0 + threadIdx.x;
    const int64_t v = j < np ? partials[j] : 0;
    int64_t tot;
    const int64_t ex = block_excl_scan(v, &tot);
    if (j < np) partials[j] = run + ex;
    run += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0 && total_out) *total_out = run;
}

template <class TIn, class TOut>
__global__ __launch_bounds__(SCAN_TPB) void k_scan_apply(const TIn* counts, int64_t nb,
                                                         const int64_t* __restrict__ partials, TOut* offsets) {
  const int64_t base = (int64_t)blockIdx.x * SCAN_CHUNK + (int64_t)threadIdx.x * SCAN_PER;   // 16 consecutive
  TIn c[SCAN_PER];
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    c[i] = base + i < nb ? counts[base + i] : 0;
    s += c[i];
  }
  int64_t tot;
  int64_t run = partials[blockIdx.x] + block_excl_scan(s, &tot);
#pragma unroll
  for (int i = 0; i < SCAN_PER; ++i) {
    if (base + i < nb) offsets[base + i] = (TOut)run;
    run += c[i];
  }
}

inline int64_t scan_partials_len(int64_t n) { return (n + SCAN_CHUNK - 1) / SCAN_CHUNK + 1; }

// out[i] = sum(in[0, i)), total -> *total_out (device, may be null); partials: scan_partials_len(n)
// int64 of device scratch
template <class TIn, class TOut>
inline void launch_excl_scan(hipStream_t s, const TIn* in, int64_t n, TOut* out, int64_t* partials,
                             int64_t* total_out) {
  const int64_t nchunks = (n + SCAN_CHUNK - 1) / SCAN_CHUNK;
  if (nchunks > 0)
    hipLaunchKernelGGL((k_scan_partials<TIn>), dim3((unsigned)nchunks), dim3(SCAN_TPB), 0, s, in, n, partials);
  hipLaunchKernelGGL(k_scan_chunks, dim3(1), dim3(SCAN_TPB), 0, s, partials, nchunks, total_out);
  if (nchunks > 0)
    hipLaunchKernelGGL((k_scan_apply<TIn, TOut>), dim3((unsigned)nchunks), dim3(SCAN_TPB), 0, s, in, n, partials, out);
}

struct ScanBufs {
  uint64_t* mask = nullptr;
  int32_t* counts = nullptr;
  int64_t* offsets = nullptr;
  int64_t* partials = nullptr;   // chunk sums of the two-level count scan
  int32_t* desc = nullptr;
};

// pass A outputs (mask words + per-block counts) and a descriptor area, carved from the context's
// scan workspace; user_mask, when given, receives the mask instead
int alloc_scan(gm_ctx* ctx, int64_t n, uint64_t* user_mask, size_t desc_words, ScanBufs& b);
void free_scan(gm_ctx* ctx, uint64_t* user_mask, ScanBufs& b);
// passes B and C: block-count scan, ids in ascending row order, match count readback
int finish_scan(gm_ctx* ctx, int64_t n, ScanBufs& b, int64_t* ids, int64_t ids_cap, int64_t* n_match);

}  // namespace gm
