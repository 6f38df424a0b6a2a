// gm_scan.hpp -- shared pieces of the mask -> block scan -> ordered compaction pipeline
// (gm_filter.hip; the fused query scan in gm_pip.hip).
#pragma once

#include "gm_internal.hpp"

namespace gm {

constexpr int FTPB = 256;             // threads per block
constexpr int FELEMS = 8;             // rows per thread per block
constexpr int FROWS = FTPB * FELEMS;  // rows per block (2048) -> 64 mask words

// ------------------------------------------------------------------ vectorised pass A
// The scalar kernels of gm_filter.hip move 2 B (bin) and 8 B (z) per lane per load instruction; on gfx950 narrow
// per-lane accesses stream at roughly half the 16-B rate.  The _v variants use the layout of the
// encode kernels: each lane takes PAIRS of consecutive rows, one 16-B load per 8-byte column
// (z, x, y, t) and one 4-B load of the two bins, and pair p of lane l in step u sits at
// block_base + u*256 + l, so every wave instruction reads one contiguous 1 KiB run.  A wave step
// covers 128 rows: ballot(row 2l) and ballot(row 2l+1) interleave bit by bit into the two 64-bit
// mask words of those rows.  A block still covers FROWS = 2048 rows (4 steps), so block_counts,
// k_scan_counts and k_mask_to_ids are shared with the scalar kernels.
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

__device__ __forceinline__ void block_count_waves(int wave_cnt, int32_t* block_counts) {
  __shared__ int s_wc[FTPB / 64];
  if ((threadIdx.x & 63) == 0) s_wc[threadIdx.x >> 6] = wave_cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < FTPB / 64; ++i) s += s_wc[i];
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

struct ScanBufs {
  uint64_t* mask = nullptr;
  int32_t* counts = nullptr;
  int64_t* offsets = nullptr;
  int32_t* desc = nullptr;
};

// pass A outputs (mask words + per-block counts) and a descriptor area, carved from the context's
// scan workspace; user_mask, when given, receives the mask instead
int alloc_scan(gm_ctx* ctx, int64_t n, uint64_t* user_mask, size_t desc_words, ScanBufs& b);
void free_scan(gm_ctx* ctx, uint64_t* user_mask, ScanBufs& b);
// passes B and C: block-count scan, ids in ascending row order, match count readback
int finish_scan(gm_ctx* ctx, int64_t n, ScanBufs& b, int64_t* ids, int64_t ids_cap, int64_t* n_match);

}  // namespace gm
