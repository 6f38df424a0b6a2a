// Gather-throughput probe (tools only, not part of the library): divergent 4-B / 16-B gathers from
// tables of different sizes (L2, Infinity Cache, HBM), random LDS reads, and a coalesced stream, so
// the join's per-point lookup costs can be priced.  Build: hipcc --offload-arch=gfx950 -O3 -o
// tools/gather_probe tools/gather_probe.hip ; run: tools/gather_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint64_t v) {
  v ^= v >> 33; v *= 0xff51afd7ed558ccdull; v ^= v >> 33; v *= 0xc4ceb9fe1a85ec53ull; v ^= v >> 33;
  return (uint32_t)v;
}

template <int U>
__global__ __launch_bounds__(256) void k_gather4(const uint32_t* __restrict__ tab, uint32_t mask, int64_t n,
                                                 unsigned long long* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[mix(i + u) & mask];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

template <int U>
__global__ __launch_bounds__(256) void k_gather16(const uint4* __restrict__ tab, uint32_t mask, int64_t n,
                                                  unsigned long long* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[mix(i + u) & mask];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].w;
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

// 8 lanes per 128-B line: lanes 8k..8k+7 read the 16-B pieces of one random line (coalesced per group)
template <int U>
__global__ __launch_bounds__(256) void k_line8(const uint4* __restrict__ tab, uint32_t lmask, int64_t n,
                                               unsigned long long* __restrict__ out) {
  uint32_t acc = 0;
  const int sub = threadIdx.x & 7;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[(uint64_t)(mix((i >> 3) * U + u) & lmask) * 8 + sub];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].w;
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

// every lane of a wave reads the same 16 B (uniform address, random per wave and step)
template <int U>
__global__ __launch_bounds__(256) void k_uniform16(const uint4* __restrict__ tab, uint32_t mask, int64_t n,
                                                   unsigned long long* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = tab[mix((i >> 6) * U + u) & mask];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].w;
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

// dependent chain: each gather's address depends on the previous value (latency, not throughput)
__global__ __launch_bounds__(256) void k_chain4(const uint32_t* __restrict__ tab, uint32_t mask, int64_t n,
                                                unsigned long long* __restrict__ out) {
  uint32_t acc = 0, a = mix(blockIdx.x * 256 + threadIdx.x);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
#pragma unroll
    for (int u = 0; u < 4; ++u) { a = tab[(a ^ mix(i + u)) & mask]; acc += a; }
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

template <int U>
__global__ __launch_bounds__(256) void k_lds4(int64_t n, unsigned long long* __restrict__ out) {
  __shared__ uint32_t t[16384];
  for (int i = threadIdx.x; i < 16384; i += 256) t[i] = mix(i);
  __syncthreads();
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = t[mix(i + u) & 16383];
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

__global__ __launch_bounds__(256) void k_stream(const double2* __restrict__ p, int64_t n, unsigned long long* out) {
  double acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = p[i];
    acc += v.x + v.y;
  }
  if (acc == 1.2345) atomicAdd(out, 1ull);
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
  const int64_t N = 1ll << 30;   // lane loads per launch
  const size_t big = (size_t)1 << 30;
  uint32_t* tab = nullptr;
  unsigned long long* out = nullptr;
  CK(hipMalloc(&tab, big));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(tab, 1, big));
  const int g = 2048;
  for (size_t tb : {(size_t)1 << 20, (size_t)64 << 20, (size_t)1 << 30}) {
    const uint32_t m16 = (uint32_t)(tb / 16 - 1), ml = (uint32_t)(tb / 128 - 1);
    float b = timeit([&] { hipLaunchKernelGGL(k_gather16<4>, dim3(g), dim3(256), 0, 0, (const uint4*)tab, m16, N, out); });
    float c = timeit([&] { hipLaunchKernelGGL(k_line8<4>, dim3(g), dim3(256), 0, 0, (const uint4*)tab, ml, N, out); });
    float d = timeit([&] { hipLaunchKernelGGL(k_uniform16<4>, dim3(g), dim3(256), 0, 0, (const uint4*)tab, m16, N, out); });
    printf("table %8zu KB (16-B lane loads): divergent %.3f ms (%.0f GB/s)  8-lane lines %.3f ms (%.0f GB/s)  uniform %.3f ms (%.0f GB/s)\n",
           tb >> 10, b, N * 16.0 / b / 1e6, c, N * 16.0 / c / 1e6, d, N * 16.0 / d / 1e6);
    fflush(stdout);
  }
  return 0;
}
