// gm_filter.hip -- fused key-space / strict filter scans with wave-ballot compaction.
//
// Z3Filter.inBounds (idx/filters/Z3Filter.scala:26-62) is evaluated for every row of a columnar
// key store in one pass: 10 B/row (bin i16 + z i64) in, 1 bit/row out.  The Scala code runs it per
// row inside RowFilterIterator (geomesa-accumulo-iterators/.../RowFilterIterator.scala:52-66) or
// Z3HBaseFilter; here a wave of 64 rows produces one 64-bit ballot word.
//
// Output pipeline (all on the context stream, deterministic, ids ascending):
//   pass A  k_*_mask     : per-row predicate -> mask words + per-block match counts
//   pass B  k_scan_counts: exclusive scan of the per-block counts (single workgroup)
//   pass C  k_mask_to_ids: expand mask bits into row ids at the scanned offsets
// Pass C reads n/8 bytes of mask, so the ids cost ~1/80 of pass A's traffic plus 8 B per match.
#include <vector>

#include "gm_internal.hpp"

namespace gm {

constexpr int FTPB = 256;             // threads per block
constexpr int FELEMS = 8;             // rows per thread per block
constexpr int FROWS = FTPB * FELEMS;  // rows per block (2048) -> 64 mask words

// ------------------------------------------------------------------ device filter descriptor
// flat int32 layout (built on the host from Z3Filter.serializeToBytes):
//   [0] nxy, [1] min_epoch, [2] max_epoch, [3] nt, [4] reserved
//   [5 .. 5+4*nxy)        xy boxes (xmin, ymin, xmax, ymax) in normalized cells
//   then nt (start, end) interval index pairs, (-1, -1) for a null epoch
//   then the intervals (t0, t1)
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

// pass B: exclusive scan of block counts by one workgroup of 1024 threads; total -> out[nb]
__global__ __launch_bounds__(1024) void k_scan_counts(const int32_t* __restrict__ counts, int64_t nb,
                                                      int64_t* __restrict__ offsets) {
  __shared__ int64_t s_part[1024];
  const int64_t per = (nb + 1023) / 1024;
  const int64_t a = (int64_t)threadIdx.x * per;
  const int64_t b = a + per < nb ? a + per : nb;
  int64_t sum = 0;
  for (int64_t i = a; i < b; ++i) sum += counts[i];
  s_part[threadIdx.x] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    int64_t v = threadIdx.x >= off ? s_part[threadIdx.x - off] : 0;
    __syncthreads();
    s_part[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t run = s_part[threadIdx.x] - sum;  // exclusive
  for (int64_t i = a; i < b; ++i) {
    offsets[i] = run;
    run += counts[i];
  }
  if (threadIdx.x == 1023) offsets[nb] = s_part[1023];
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

// ------------------------------------------------------------------ host side

static inline int32_t be32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | (uint32_t)p[3]);
}
static inline int16_t be16(const uint8_t* p) { return (int16_t)(uint16_t)((uint16_t)p[0] << 8 | p[1]); }

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

namespace {

struct ScanBufs {
  uint64_t* mask = nullptr;
  int32_t* counts = nullptr;
  int64_t* offsets = nullptr;
  int32_t* desc = nullptr;
};

// scratch buffers per call (hipMallocAsync keeps them stream-ordered)
int alloc_scan(gm_ctx* ctx, int64_t n, uint64_t* user_mask, size_t desc_words, ScanBufs& b) {
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  const int64_t nwords = nblocks * (FROWS / 64);
  if (!user_mask) GM_HIP(hipMallocAsync((void**)&b.mask, (size_t)nwords * 8, ctx->stream));
  else b.mask = (uint64_t*)user_mask;
  GM_HIP(hipMallocAsync((void**)&b.counts, (size_t)nblocks * 4 + 4, ctx->stream));
  GM_HIP(hipMallocAsync((void**)&b.offsets, (size_t)(nblocks + 1) * 8, ctx->stream));
  if (desc_words) GM_HIP(hipMallocAsync((void**)&b.desc, desc_words * 4, ctx->stream));
  return GM_OK;
}

void free_scan(gm_ctx* ctx, uint64_t* user_mask, ScanBufs& b) {
  if (!user_mask && b.mask) (void)hipFreeAsync(b.mask, ctx->stream);
  if (b.counts) (void)hipFreeAsync(b.counts, ctx->stream);
  if (b.offsets) (void)hipFreeAsync(b.offsets, ctx->stream);
  if (b.desc) (void)hipFreeAsync(b.desc, ctx->stream);
}

// passes B and C + count readback
int finish_scan(gm_ctx* ctx, int64_t n, ScanBufs& b, int64_t* ids, int64_t ids_cap, int64_t* n_match) {
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  if (ids || n_match) {
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, ctx->stream, b.counts, nblocks, b.offsets);
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
  ScanBufs b;
  int rc = alloc_scan(ctx, n, mask, desc.size(), b);
  if (rc) return rc;
  GM_HIP(hipMemcpyAsync(b.desc, desc.data(), desc.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));  // desc is pageable host memory
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  const size_t lds = desc.size() * 4;
  hipLaunchKernelGGL(k_z3filter_mask, dim3((unsigned)nblocks), dim3(FTPB), lds, ctx->stream, bin, z, n, b.desc, fwords,
                     b.desc + fwords, n_bin_ranges, b.mask, b.counts);
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
  ScanBufs b;
  int rc = alloc_scan(ctx, n, mask, xy.size() + 1, b);
  if (rc) return rc;
  if (!xy.empty()) GM_HIP(hipMemcpyAsync(b.desc, xy.data(), xy.size() * 4, hipMemcpyHostToDevice, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  const int64_t nblocks = (n + FROWS - 1) / FROWS;
  hipLaunchKernelGGL(k_z2filter_mask, dim3((unsigned)nblocks), dim3(FTPB), xy.size() * 4 + 4, ctx->stream, z, n,
                     b.desc, nxy, b.mask, b.counts);
  GM_CHECK_LAUNCH();
  rc = finish_scan(ctx, n, b, ids, ids_cap, n_match);
  free_scan(ctx, mask, b);
  if (rc) return rc;
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
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
  if (has_during)
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

}  // extern "C"
