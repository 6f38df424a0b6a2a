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
  char* h_stage = nullptr;         // pinned staging for copies to / from pageable host memory (2 halves)
  void* ws[4] = {nullptr, nullptr, nullptr, nullptr};   // reusable device workspaces (see ctx_workspace)
  size_t ws_cap[4] = {0, 0, 0, 0};
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int64_t join_chunk = 0;          // GM_PARAM_JOIN_CHUNK: rows per join pass (0 = default, 2^31)
  int64_t index_build = 0;         // GM_PARAM_INDEX_BUILD: 0 = device build of the join index, 1 = host build
  int64_t ranges_hint = 0;         // largest batched-ranges output seen (sizes the device batch buffer)
  int64_t ranges_chunk = 0;        // GM_PARAM_RANGES_CHUNK: queries per pipelined chunk (0 = default)
  int64_t sort_last = 0;           // GM_PARAM_SORT_LAST (read-only): the last sort's digit passes | 256 if ranked locally
  int64_t sort_mode = 0;           // GM_PARAM_SORT_MODE: 0 = auto (prefix passes + local ranks), 1 = digit passes only
  int64_t index_coarse = -1;       // GM_PARAM_INDEX_COARSE: the join's coarse sub-block masks (-1 = automatic)
  int64_t hist_grid = 0;           // GM_PARAM_HIST_GRID: Z3Histogram LDS-kernel workgroups (0 = default)
  int64_t relate_rows64 = 0;       // GM_PARAM_RELATE_ROWS64: the row predicate's 64-bit-row kernel always
  uint32_t fault_calls = 0;        // FC_* bits: the entry points that enqueued reference-checked kernels
                                   // since the fault word was last read (take_fault names them)
  hipStream_t copy_stream = nullptr;   // result copies overlapping the next chunk's kernels (lazy)
  hipEvent_t ev_ready[2] = {nullptr, nullptr}, ev_copied[2] = {nullptr, nullptr};
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

// Host <-> device copies of caller host memory.  Pinned (hipHostMalloc'd / registered) memory is
// copied directly; pageable memory goes through the context's pinned staging buffer in
// double-buffered pieces (direct DMA to pageable memory degrades badly on this stack: a 256 MB
// result copy took 0.3-7 s and grew from call to call, against 80 ms through pinned memory).
// Both synchronise the context stream.
int copy_d2h(gm_ctx* ctx, void* host, const void* dev, size_t bytes);
int copy_h2d(gm_ctx* ctx, void* dev, const void* host, size_t bytes);

// A device workspace owned by the context, grown on demand and reused by later calls (calls on
// one context are stream-ordered, so reuse is safe).  Large per-call temporaries come from here
// rather than hipMallocAsync: on this stack multi-GB pool allocations were re-mapped on every call
// (0.7-6 s stalls between launches).  slot: 0 = range batches, 1 = sort, 2 = scans, 3 = join.
enum : int { WS_RANGES = 0, WS_SORT = 1, WS_SCAN = 2, WS_JOIN = 3 };
int ctx_workspace(gm_ctx* ctx, int slot, size_t bytes, void** p);
bool host_pinned(const void* p);
bool device_memory(const void* p);   // device (hipMalloc) memory, as opposed to host memory
int ctx_copy_stream(gm_ctx* ctx);   // creates copy_stream and its events on first use

// The context's sticky reference-fault word (d_scratch[SCRATCH_FAULT]): the polygon-index kernels OR
// PIP_FAULT_* bits into it, stream-ordered; take_fault (a synchronising call: a join that returns its
// pair count, a query scan, gm_ctx_sync) reads and clears it and returns GM_E_INDEX when set.
// A stream-ordered call (gm_pip_relate, a join without n_pairs) leaves its bits for a later
// synchronising call, so each call that enqueues checked kernels records itself (note_fault_call) and
// the error text names every such call since the last read, not only the call that read the word.
constexpr int SCRATCH_FAULT = 63;
enum : uint32_t { FC_JOIN = 1, FC_JOIN_ARROW = 2, FC_RELATE = 4, FC_QUERY = 8 };
inline void note_fault_call(gm_ctx* ctx, uint32_t fc) { ctx->fault_calls |= fc; }
int take_fault(gm_ctx* ctx, const char* what);

// reset the error summary before a call that reports one
int begin_summary(gm_ctx* ctx, gm_batch_status* summary);
// read the summary back (synchronises the stream); maps to GM_OK / per-element semantics
int end_summary(gm_ctx* ctx, gm_batch_status* summary);

// Resident block count of `kernel` at `block` threads per block on `device`: occupancy x CUs,
// computed once per (kernel, device) under a lock (contexts on different devices and concurrent
// callers are safe); `fallback_per_cu` when the occupancy query fails.
int resident_blocks(const void* kernel, int device, int block, int fallback_per_cu);

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

inline unsigned grid_for(int64_t n, int64_t per_block) {
  int64_t b = (n + per_block - 1) / per_block;
  return (unsigned)(b < 1 ? 1 : b);
}

}  // namespace gm
