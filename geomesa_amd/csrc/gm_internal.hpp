// gm_internal.hpp -- context, error plumbing and launch helpers shared by the libgeomesa_hip units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/geomesa_hip.h"
#include "gm_device.hpp"

struct gm_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int64_t* d_err = nullptr;        // [0] error count, [1] packed (first index << 8 | code)
  int64_t* d_scratch = nullptr;    // small device scratch: counters
  int64_t* h_pinned = nullptr;     // pinned host mirror for summaries / counters
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};

namespace gm {

void set_error(const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define GM_HIP(expr)                                   \
  do {                                                 \
    hipError_t _e = (expr);                            \
    if (_e != hipSuccess) return gm::hip_fail(_e, #expr); \
  } while (0)

#define GM_CHECK_LAUNCH() GM_HIP(hipGetLastError())

// device-side element error report: called only by failing lanes (rare path)
__device__ __forceinline__ void report_error(int64_t* err, int64_t idx, uint8_t code) {
  atomicAdd((unsigned long long*)&err[0], 1ull);
  atomicMin((long long*)&err[1], (long long)((idx << 8) | code));
}

// reset the error summary before a call that reports one
int begin_summary(gm_ctx* ctx, gm_batch_status* summary);
// read the summary back (synchronises the stream); maps to GM_OK / per-element semantics
int end_summary(gm_ctx* ctx, gm_batch_status* summary);

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

inline unsigned grid_for(int64_t n, int64_t per_block) {
  int64_t b = (n + per_block - 1) / per_block;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace gm
