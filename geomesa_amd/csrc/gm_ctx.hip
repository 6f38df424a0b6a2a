// gm_ctx.hip -- context lifecycle, error plumbing, memory helpers, timers, synthetic data.
#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "gm_internal.hpp"

namespace {
thread_local std::string g_last_error;
}

namespace gm {

constexpr size_t STAGE_HALF = (size_t)16 << 20;   // two 16 MiB halves

static bool is_pinned(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();   // unregistered pageable memory reports an error: clear it
    return false;
  }
  return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

int resident_blocks(const void* kernel, int device, int block, int fallback_per_cu) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair(kernel, device);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int b = 0, cus = 256, prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kernel, block, 0) != hipSuccess || b < 1) {
    (void)hipGetLastError();
    b = fallback_per_cu;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus = prop.multiProcessorCount;
  (void)hipSetDevice(prev);
  const int r = std::max(1, b * cus);
  cache[key] = r;
  return r;
}

static int stage(gm_ctx* ctx) {
  if (!ctx->h_stage) GM_HIP(hipHostMalloc((void**)&ctx->h_stage, 2 * STAGE_HALF, hipHostMallocDefault));
  return GM_OK;
}

int copy_d2h(gm_ctx* ctx, void* host, const void* dev, size_t bytes) {
  if (!bytes) return GM_OK;
  if (bytes <= 4096 || is_pinned(host)) {
    GM_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    return GM_OK;
  }
  int rc = stage(ctx);
  if (rc) return rc;
  // piece k lands in half k % 2; piece k's host copy overlaps piece k + 1's DMA
  const char* src = (const char*)dev;
  char* dst = (char*)host;
  size_t off = 0, prev_off = 0, prev_len = 0;
  int k = 0;
  while (off < bytes || prev_len) {
    size_t len = 0;
    if (off < bytes) {
      len = std::min(STAGE_HALF, bytes - off);
      GM_HIP(hipMemcpyAsync(ctx->h_stage + (k % 2) * STAGE_HALF, src + off, len, hipMemcpyDeviceToHost, ctx->stream));
    }
    if (prev_len) memcpy(dst + prev_off, ctx->h_stage + ((k + 1) % 2) * STAGE_HALF, prev_len);
    GM_HIP(hipStreamSynchronize(ctx->stream));
    prev_off = off; prev_len = len; off += len; ++k;
  }
  return GM_OK;
}

bool host_pinned(const void* p) { return is_pinned(p); }

bool device_memory(const void* p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

int ctx_copy_stream(gm_ctx* ctx) {
  if (ctx->copy_stream) return GM_OK;
  GM_HIP(hipSetDevice(ctx->device));
  GM_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  for (int k = 0; k < 2; ++k) {
    GM_HIP(hipEventCreateWithFlags(&ctx->ev_ready[k], hipEventDisableTiming));
    GM_HIP(hipEventCreateWithFlags(&ctx->ev_copied[k], hipEventDisableTiming));
  }
  return GM_OK;
}

int ctx_workspace(gm_ctx* ctx, int slot, size_t bytes, void** p) {
  if (ctx->ws_cap[slot] < bytes) {
    GM_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->ws[slot]) GM_HIP(hipFree(ctx->ws[slot]));
    ctx->ws[slot] = nullptr;
    ctx->ws_cap[slot] = 0;
    const size_t want = (bytes + bytes / 4 + 4095) & ~(size_t)4095;
    GM_HIP(hipMalloc(&ctx->ws[slot], want));
    ctx->ws_cap[slot] = want;
  }
  *p = ctx->ws[slot];
  return GM_OK;
}

int copy_h2d(gm_ctx* ctx, void* dev, const void* host, size_t bytes) {
  if (!bytes) return GM_OK;
  if (bytes <= 4096 || is_pinned(host)) {
    GM_HIP(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    return GM_OK;
  }
  int rc = stage(ctx);
  if (rc) return rc;
  const char* src = (const char*)host;
  char* dst = (char*)dev;
  for (size_t off = 0; off < bytes; off += STAGE_HALF) {
    const size_t len = std::min(STAGE_HALF, bytes - off);
    memcpy(ctx->h_stage, src + off, len);
    GM_HIP(hipMemcpyAsync(dst + off, ctx->h_stage, len, hipMemcpyHostToDevice, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
  }
  return GM_OK;
}


void set_error(const std::string& msg) { g_last_error = msg; }

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return GM_E_HIP;
}

int begin_summary(gm_ctx* ctx, gm_batch_status* summary) {
  if (!summary) return GM_OK;
  const int64_t init[2] = {0, INT64_MAX};
  GM_HIP(hipMemcpyAsync(ctx->d_err, init, sizeof(init), hipMemcpyHostToDevice, ctx->stream));
  return GM_OK;
}

int end_summary(gm_ctx* ctx, gm_batch_status* summary) {
  if (!summary) return GM_OK;
  GM_HIP(hipMemcpyAsync(ctx->h_pinned, ctx->d_err, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  GM_HIP(hipStreamSynchronize(ctx->stream));
  summary->n_errors = ctx->h_pinned[0];
  if (ctx->h_pinned[0] > 0) {
    summary->first_index = ctx->h_pinned[1] >> 8;
    summary->first_code = (int32_t)(ctx->h_pinned[1] & 0xff);
  } else {
    summary->first_index = -1;
    summary->first_code = 0;
  }
  summary->reserved = 0;
  return GM_OK;
}

// SplitMix64 (Steele, Lea, Flood 2014), keyed by (seed, index)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ double unit_double(uint64_t r) { return (double)(r >> 11) * 0x1.0p-53; }

__global__ __launch_bounds__(256) void k_gen_points(uint64_t seed, int64_t n, int64_t base, double lon0,
                                                    double lon1, double lat0, double lat1, int64_t t0,
                                                    int64_t t1, double* __restrict__ x, double* __restrict__ y,
                                                    int64_t* __restrict__ t) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t k = (uint64_t)(base + i);
  uint64_t r0 = splitmix64(seed ^ (k * 3 + 0) * 0xd1b54a32d192ed03ull);
  uint64_t r1 = splitmix64(seed ^ (k * 3 + 1) * 0xd1b54a32d192ed03ull);
  uint64_t r2 = splitmix64(seed ^ (k * 3 + 2) * 0xd1b54a32d192ed03ull);
  if (x) x[i] = __dadd_rn(lon0, __dmul_rn(unit_double(r0), __dsub_rn(lon1, lon0)));
  if (y) y[i] = __dadd_rn(lat0, __dmul_rn(unit_double(r1), __dsub_rn(lat1, lat0)));
  if (t) {
    uint64_t span = (uint64_t)(t1 - t0);
    t[i] = t0 + (int64_t)(span ? (r2 % span) : 0);
  }
}

// Device-to-device stream copy: 16 B per lane, four vectors per lane in flight, non-temporal loads and
// stores (the access shape of the encode kernels), one-shot blocks.  The streaming ceiling the bench
// measures the box against (torch's copy_ of bytes ran slower than the encode kernel itself).
constexpr int CPY_U = 4;
__global__ __launch_bounds__(256) void k_stream_copy(const lv2* __restrict__ src, lv2* __restrict__ dst, int64_t nv) {
  const int64_t base = (int64_t)blockIdx.x * (256 * CPY_U) + threadIdx.x;
  lv2 v[CPY_U];
  if (base + (CPY_U - 1) * 256 < nv) {   // a full block: unconditional loads, all in flight together
#pragma unroll
    for (int u = 0; u < CPY_U; ++u) v[u] = __builtin_nontemporal_load(&src[base + u * 256]);
#pragma unroll
    for (int u = 0; u < CPY_U; ++u) __builtin_nontemporal_store(v[u], &dst[base + u * 256]);
  } else {
#pragma unroll
    for (int u = 0; u < CPY_U; ++u)
      if (base + u * 256 < nv) __builtin_nontemporal_store(__builtin_nontemporal_load(&src[base + u * 256]), &dst[base + u * 256]);
  }
}

}  // namespace gm

namespace gm {
int take_fault(gm_ctx* c, const char* what) {
  int64_t bits = 0;
  GM_HIP(hipMemcpyAsync(c->h_pinned + 63, c->d_scratch + SCRATCH_FAULT, 8, hipMemcpyDeviceToHost, c->stream));
  GM_HIP(hipStreamSynchronize(c->stream));
  bits = c->h_pinned[63];
  const uint32_t calls = c->fault_calls;
  c->fault_calls = 0;
  if (!bits) return GM_OK;
  GM_HIP(hipMemsetAsync(c->d_scratch + SCRATCH_FAULT, 0, 8, c->stream));
  std::string src;
  const char* names[4] = {"gm_pip_join", "gm_pip_join_arrow", "gm_pip_relate", "gm_query_scan"};
  for (int k = 0; k < 4; ++k)
    if (calls & (1u << k)) src += std::string(src.empty() ? "" : ", ") + names[k];
  char msg[400];
  snprintf(msg, sizeof msg, "%s: device reference check failed (PIP_FAULT bits 0x%x): corrupt index or internal "
           "queue invariant; raised by a kernel of one of the calls on this context since the last check "
           "(stream-ordered calls report here): %s", what, (unsigned)bits, src.empty() ? "unknown" : src.c_str());
  set_error(msg);
  return GM_E_INDEX;
}
}  // namespace gm


extern "C" {

int gm_abi_version(void) { return GM_ABI_VERSION; }

const char* gm_last_error(void) { return g_last_error.c_str(); }

static int ctx_create(int device, void* stream, bool own, gm_ctx** out) {
  if (!out) return GM_E_INVALID;
  *out = nullptr;
  int ndev = 0;
  GM_HIP(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    gm::set_error("gm_ctx_create: no such device");
    return GM_E_INVALID;
  }
  GM_HIP(hipSetDevice(device));
  gm_ctx* c = new gm_ctx();
  c->device = device;
  if (!own) {
    c->stream = (hipStream_t)stream;  // NULL = the device's default (null) stream
  } else {
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return gm::hip_fail(e, "hipStreamCreate"); }
    c->own_stream = true;
  }
  hipError_t e = hipMalloc(&c->d_err, 4 * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&c->d_scratch, 64 * sizeof(int64_t));
  if (e == hipSuccess) e = hipMemset(c->d_scratch, 0, 64 * sizeof(int64_t));
  if (e == hipSuccess) e = hipHostMalloc(&c->h_pinned, 64 * sizeof(int64_t), hipHostMallocDefault);
  if (e == hipSuccess) e = hipEventCreate(&c->ev0);
  if (e == hipSuccess) e = hipEventCreate(&c->ev1);
  if (e != hipSuccess) { gm_ctx_destroy(c); return gm::hip_fail(e, "gm_ctx_create"); }
  // The scans, sort, partitioned join and range batches take their temporaries with
  // hipMallocAsync.  With the pool's default release threshold (0) every synchronisation hands the
  // memory back and the next call maps it again (seconds for multi-GB range workspaces), so the
  // device's default pool keeps what it has reserved, as a caching allocator does.
  hipMemPool_t pool = nullptr;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess && pool) {
    uint64_t keep = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  }
  *out = c;
  return GM_OK;
}

int gm_ctx_create(int device, void* stream, gm_ctx** out) { return ctx_create(device, stream, false, out); }

int gm_ctx_create_owned(int device, gm_ctx** out) { return ctx_create(device, nullptr, true, out); }

int gm_ctx_destroy(gm_ctx* c) {
  if (!c) return GM_OK;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->d_err) (void)hipFree(c->d_err);
  if (c->d_scratch) (void)hipFree(c->d_scratch);
  if (c->h_pinned) (void)hipHostFree(c->h_pinned);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  for (void* w : c->ws)
    if (w) (void)hipFree(w);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  for (int k = 0; k < 2; ++k) {
    if (c->ev_ready[k]) (void)hipEventDestroy(c->ev_ready[k]);
    if (c->ev_copied[k]) (void)hipEventDestroy(c->ev_copied[k]);
  }
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GM_OK;
}

int gm_ctx_sync(gm_ctx* c) {
  if (!c) return GM_E_INVALID;
  GM_HIP(hipStreamSynchronize(c->stream));
  return gm::take_fault(c, "gm_ctx_sync");
}

void* gm_ctx_stream(gm_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gm_ctx_set_param(gm_ctx* c, int param, int64_t value) {
  if (!c) return GM_E_INVALID;
  switch (param) {
    case GM_PARAM_JOIN_CHUNK:
      if (value < 0) return GM_E_INVALID;
      c->join_chunk = value;
      return GM_OK;
    case GM_PARAM_INDEX_BUILD:
      if (value != 0 && value != 1) return GM_E_INVALID;
      c->index_build = value;
      return GM_OK;
    case GM_PARAM_RANGES_CHUNK:
      if (value < 0) return GM_E_INVALID;
      c->ranges_chunk = value;
      return GM_OK;
    case GM_PARAM_SORT_MODE:
      if (value != 0 && value != 1) return GM_E_INVALID;
      c->sort_mode = value;
      return GM_OK;
    case GM_PARAM_INDEX_COARSE:
      if (value < -1 || value > 1) return GM_E_INVALID;
      c->index_coarse = value;
      return GM_OK;
    case GM_PARAM_HIST_GRID:
      if (value < 0 || value > (1 << 20)) return GM_E_INVALID;
      c->hist_grid = value;
      return GM_OK;
    case GM_PARAM_RELATE_ROWS64:
      if (value != 0 && value != 1) return GM_E_INVALID;
      c->relate_rows64 = value;
      return GM_OK;
    case GM_PARAM_INDEX_CORE_RETIRED:   // retired in round 5: accepted, ignored (one release)
      return GM_OK;
    default:
      gm::set_error("gm_ctx_set_param: unknown parameter");
      return GM_E_INVALID;
  }
}

int gm_ctx_get_param(gm_ctx* c, int param, int64_t* value) {
  if (!c || !value) return GM_E_INVALID;
  switch (param) {
    case GM_PARAM_JOIN_CHUNK: *value = c->join_chunk; return GM_OK;
    case GM_PARAM_INDEX_BUILD: *value = c->index_build; return GM_OK;
    case GM_PARAM_RANGES_CHUNK: *value = c->ranges_chunk; return GM_OK;
    case GM_PARAM_SORT_MODE: *value = c->sort_mode; return GM_OK;
    case GM_PARAM_SORT_LAST: *value = c->sort_last; return GM_OK;
    case GM_PARAM_INDEX_COARSE: *value = c->index_coarse; return GM_OK;
    case GM_PARAM_HIST_GRID: *value = c->hist_grid; return GM_OK;
    case GM_PARAM_INDEX_CORE_RETIRED: *value = 0; return GM_OK;
    case GM_PARAM_RELATE_ROWS64: *value = c->relate_rows64; return GM_OK;
    default: return GM_E_INVALID;
  }
}

int gm_device_alloc(gm_ctx* c, size_t bytes, void** ptr) {
  if (!c || !ptr) return GM_E_INVALID;
  GM_HIP(hipSetDevice(c->device));
  GM_HIP(hipMalloc(ptr, bytes ? bytes : 1));
  return GM_OK;
}
int gm_device_free(gm_ctx* c, void* ptr) {
  if (!c) return GM_E_INVALID;
  if (ptr) GM_HIP(hipFree(ptr));
  return GM_OK;
}
int gm_copy_to_device(gm_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c || (bytes && (!dst || !src))) return GM_E_INVALID;
  return gm::copy_h2d(c, dst, src, bytes);
}
int gm_copy_to_host(gm_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c || (bytes && (!dst || !src))) return GM_E_INVALID;
  return gm::copy_d2h(c, dst, src, bytes);
}
int gm_device_copy(gm_ctx* c, void* dst, const void* src, size_t bytes) {
  if (!c || (bytes && (!dst || !src))) return GM_E_INVALID;
  if (!bytes) return GM_OK;
  size_t head = 0;
  if (gm::aligned16(dst) && gm::aligned16(src) && bytes >= 16) {
    const int64_t nv = (int64_t)(bytes / 16);
    head = (size_t)nv * 16;
    hipLaunchKernelGGL(gm::k_stream_copy, dim3((unsigned)((nv + 256 * gm::CPY_U - 1) / (256 * gm::CPY_U))), dim3(256), 0,
                       c->stream, (const gm::lv2*)src, (gm::lv2*)dst, nv);
    GM_CHECK_LAUNCH();
  }
  if (head < bytes)
    GM_HIP(hipMemcpyAsync((char*)dst + head, (const char*)src + head, bytes - head, hipMemcpyDeviceToDevice, c->stream));
  return GM_OK;
}
int gm_timer_start(gm_ctx* c) {
  if (!c) return GM_E_INVALID;
  GM_HIP(hipEventRecord(c->ev0, c->stream));
  return GM_OK;
}
int gm_timer_stop(gm_ctx* c, float* ms) {
  if (!c || !ms) return GM_E_INVALID;
  GM_HIP(hipEventRecord(c->ev1, c->stream));
  GM_HIP(hipEventSynchronize(c->ev1));
  GM_HIP(hipEventElapsedTime(ms, c->ev0, c->ev1));
  return GM_OK;
}

int gm_gen_points(gm_ctx* c, uint64_t seed, int64_t n, int64_t base, double lon0, double lon1, double lat0,
                  double lat1, int64_t t0, int64_t t1, double* x, double* y, int64_t* t) {
  if (!c || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  hipLaunchKernelGGL(gm::k_gen_points, dim3(gm::grid_for(n, 256)), dim3(256), 0, c->stream, seed, n, base, lon0,
                     lon1, lat0, lat1, t0, t1, x, y, t);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

}  // extern "C"
