// HBM-traffic calibration probe (tools only, not part of the library): access patterns whose bytes are
// known, so rocprofv3's memory-side read counters can be checked against them before they are used as
// the bench's `roofline.traffic` for kernels that gather.  Every table is 4 GiB (past the 256 MiB
// Infinity Cache), every pattern is its own kernel (one PMC row each):
//   k_tp_stream_read  16 B per lane, coalesced, each byte once          known: 4 GiB read
//   k_tp_copy         16 B per lane read + 16 B per lane store           known: 2 GiB read + 2 GiB written
//   k_tp_line_once    8 lanes x 16 B = one whole 128-B line, every line once, lines in a permuted order
//                                                                       known: 4 GiB read
//   k_tp_word_once    one lane reads 4 B of a line, every line once, permuted: 2^25 misses, one per line
//   k_tp_half_once    two lanes read 4 B at offsets 0 and 64 of one line (same instruction), permuted
//   k_tp_gather4 / 8 / 16   2^28 random 4-B / 8-B / 16-B reads (the join's index gathers)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/traffic_probe tools/traffic_probe.hip
// Run under rocprofv3 --pmc with TCC_EA0_RDREQ{,_32B,_64B,_128B}_sum, FETCH_SIZE, WRITE_SIZE passes.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef long long lv2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t mix(uint64_t v) {
  v ^= v >> 33; v *= 0xff51afd7ed558ccdull; v ^= v >> 33; v *= 0xc4ceb9fe1a85ec53ull; v ^= v >> 33;
  return (uint32_t)v;
}
constexpr uint64_t PERM = 0x9E3779B1ull;   // odd: i -> i * PERM mod 2^k is a permutation of the lines

__global__ __launch_bounds__(256) void k_tp_stream_read(const lv2* __restrict__ p, int64_t nv, unsigned long long* out) {
  long long acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < nv; i += stride) {
    lv2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = i + u * 256 < nv ? p[i + u * 256] : lv2{0, 0};
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y;
  }
  if (acc == 0x123456789ll) atomicAdd(out, 1ull);
}

__global__ __launch_bounds__(256) void k_tp_copy(const lv2* __restrict__ p, lv2* __restrict__ q, int64_t nv) {
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < nv; i += stride) {
    lv2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * 256 < nv) v[u] = p[i + u * 256];
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * 256 < nv) q[i + u * 256] = v[u];
  }
}

// lanes 8k..8k+7 read the 16-B pieces of line perm(j): every line exactly once
__global__ __launch_bounds__(256) void k_tp_line_once(const lv2* __restrict__ p, int64_t nlines, unsigned long long* out) {
  long long acc = 0;
  const int sub = threadIdx.x & 7;
  const uint64_t mask = (uint64_t)nlines - 1;
  const int64_t groups = (int64_t)gridDim.x * 32;
  for (int64_t j = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3); j < nlines; j += groups) {
    const uint64_t line = ((uint64_t)j * PERM) & mask;
    const lv2 v = p[line * 8 + sub];
    acc ^= v.x ^ v.y;
  }
  if (acc == 0x123456789ll) atomicAdd(out, 1ull);
}

// one lane per line: 4 B at offset 0 of line perm(j), every line exactly once
__global__ __launch_bounds__(256) void k_tp_word_once(const uint32_t* __restrict__ p, int64_t nlines, unsigned long long* out) {
  uint32_t acc = 0;
  const uint64_t mask = (uint64_t)nlines - 1;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < nlines; j += (int64_t)gridDim.x * 256) {
    const uint64_t line = ((uint64_t)j * PERM) & mask;
    acc ^= p[line * 32];
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

// two adjacent lanes per line: 4 B at offsets 0 and 64 of line perm(j)
__global__ __launch_bounds__(256) void k_tp_half_once(const uint32_t* __restrict__ p, int64_t nlines, unsigned long long* out) {
  uint32_t acc = 0;
  const uint64_t mask = (uint64_t)nlines - 1;
  const int half = threadIdx.x & 1;
  const int64_t groups = (int64_t)gridDim.x * 128;
  for (int64_t j = (int64_t)blockIdx.x * 128 + (threadIdx.x >> 1); j < nlines; j += groups) {
    const uint64_t line = ((uint64_t)j * PERM) & mask;
    acc ^= p[line * 32 + half * 16];
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

template <class T>
__global__ __launch_bounds__(256) void k_tp_gather(const T* __restrict__ p, uint64_t mask, int64_t n, unsigned long long* out) {
  uint64_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256 * 4;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += stride) {
    T v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[mix(i + u) & mask];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= (uint64_t)*(const uint32_t*)&v[u];
  }
  if (acc == 0x12345678ull) atomicAdd(out, 1ull);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <class F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 3; ++r) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 3;
}

int main() {
  const size_t big = (size_t)4 << 30;
  char* tab = nullptr;
  char* dst = nullptr;
  unsigned long long* out = nullptr;
  CK(hipMalloc(&tab, big));
  CK(hipMalloc(&dst, big / 2));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(tab, 1, big));
  const int g = 2048;
  const int64_t nv = big / 16, nlines = big / 128, ng = (int64_t)1 << 28;
  float t;
  t = timeit([&] { hipLaunchKernelGGL(k_tp_stream_read, dim3(g), dim3(256), 0, 0, (const lv2*)tab, nv, out); });
  printf("stream_read  %.3f ms  4 GiB read: %.0f GB/s\n", t, big / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_copy, dim3(g), dim3(256), 0, 0, (const lv2*)tab, (lv2*)dst, nv / 2); });
  printf("copy         %.3f ms  2 GiB + 2 GiB: %.0f GB/s\n", t, big / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_line_once, dim3(g), dim3(256), 0, 0, (const lv2*)tab, nlines, out); });
  printf("line_once    %.3f ms  %lld whole lines: %.0f GB/s of lines\n", t, (long long)nlines, big / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_word_once, dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, nlines, out); });
  printf("word_once    %.3f ms  %lld lines, 4 B each: %.2f G lines/s\n", t, (long long)nlines, nlines / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_half_once, dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, nlines, out); });
  printf("half_once    %.3f ms  %lld lines, 4 B at 0 and 64: %.2f G lines/s\n", t, (long long)nlines, nlines / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_gather<uint32_t>, dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, (uint64_t)(big / 4 - 1), ng, out); });
  printf("gather4      %.3f ms  %lld random 4-B reads: %.1f G/s\n", t, (long long)ng, ng / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_gather<uint64_t>, dim3(g), dim3(256), 0, 0, (const uint64_t*)tab, (uint64_t)(big / 8 - 1), ng, out); });
  printf("gather8      %.3f ms  %lld random 8-B reads: %.1f G/s\n", t, (long long)ng, ng / t / 1e6);
  t = timeit([&] { hipLaunchKernelGGL(k_tp_gather<lv2>, dim3(g), dim3(256), 0, 0, (const lv2*)tab, (uint64_t)(big / 16 - 1), ng, out); });
  printf("gather16     %.3f ms  %lld random 16-B reads: %.1f G/s\n", t, (long long)ng, ng / t / 1e6);
  fflush(stdout);
  return 0;
}
