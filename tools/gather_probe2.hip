// Gather-policy probe (tools only, not part of the library): divergent 4-B gathers from tables of
// 1 MiB .. 1 GiB with the default cache policy, non-temporal loads (nt) and L1-bypassing agent-scope
// loads (sc1), plus 2-B and 1-B gathers, to price what one random table lookup of the join costs at
// each level of the hierarchy.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/gather_probe2
// tools/gather_probe2.hip ; run: tools/gather_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint64_t v) {
  v ^= v >> 33; v *= 0xff51afd7ed558ccdull; v ^= v >> 33; v *= 0xc4ceb9fe1a85ec53ull; v ^= v >> 33;
  return (uint32_t)v;
}

// POL 0 = plain, 1 = nontemporal, 2 = agent-scope relaxed atomic load (sc1: bypasses L1)
template <int POL, class T>
__device__ __forceinline__ T ld(const T* p) {
  if (POL == 1) return __builtin_nontemporal_load(p);
  if (POL == 2) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

template <int POL, class T, int U>
__global__ __launch_bounds__(256) void k_gather(const T* __restrict__ tab, uint32_t mask, int64_t n,
                                                unsigned long long* __restrict__ out) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * U; i < n; i += stride) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<POL>(tab + (mix(i + u) & mask));
#pragma unroll
    for (int u = 0; u < U; ++u) acc += (uint32_t)v[u];
  }
  if (acc == 0x12345678u) atomicAdd(out, 1ull);
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
  const int64_t N = 1ll << 29;   // lane loads per launch
  const size_t big = (size_t)1 << 30;
  char* tab = nullptr;
  unsigned long long* out = nullptr;
  CK(hipMalloc(&tab, big));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(tab, 1, big));
  const int g = 4096;
  for (size_t tb : {(size_t)1 << 20, (size_t)2 << 20, (size_t)4 << 20, (size_t)16 << 20, (size_t)64 << 20, (size_t)1 << 30}) {
    const uint32_t m4 = (uint32_t)(tb / 4 - 1), m2 = (uint32_t)(tb / 2 - 1), m1 = (uint32_t)(tb - 1);
    const float p = timeit([&] { hipLaunchKernelGGL((k_gather<0, uint32_t, 4>), dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, m4, N, out); });
    const float t = timeit([&] { hipLaunchKernelGGL((k_gather<1, uint32_t, 4>), dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, m4, N, out); });
    const float s = timeit([&] { hipLaunchKernelGGL((k_gather<2, uint32_t, 4>), dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, m4, N, out); });
    const float h = timeit([&] { hipLaunchKernelGGL((k_gather<0, uint16_t, 4>), dim3(g), dim3(256), 0, 0, (const uint16_t*)tab, m2, N, out); });
    const float b = timeit([&] { hipLaunchKernelGGL((k_gather<0, uint8_t, 4>), dim3(g), dim3(256), 0, 0, (const uint8_t*)tab, m1, N, out); });
    const float s8 = timeit([&] { hipLaunchKernelGGL((k_gather<0, uint32_t, 8>), dim3(g), dim3(256), 0, 0, (const uint32_t*)tab, m4, N, out); });
    printf("table %8zu KB: 4B plain %.1f G/s  nt %.1f  sc1 %.1f  | 2B plain %.1f  1B plain %.1f | 4B plain x8 in flight %.1f\n",
           tb >> 10, N / p / 1e6, N / t / 1e6, N / s / 1e6, N / h / 1e6, N / b / 1e6, N / s8 / 1e6);
    fflush(stdout);
  }
  return 0;
}
