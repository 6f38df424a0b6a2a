// gm_pip_query.hip -- the fused point-query filter: BBOX AND during AND the OR over query polygons
// (INTERSECTS / CONTAINS), in one pass over the columns, using a polygon index (gm_pip.hpp) for
// the geometry term.  Reference: Z3IndexKeySpace.scala:240-254 (useFullFilter),
// GeometryProcessing.scala:104-136, FastTemporalOperator.scala:116-129.
#include "gm_pip.hpp"
#include "gm_scan.hpp"

namespace gm {

// ------------------------------------------------------------------ fused query scan
// The full filter of a point query in one pass over the columns (Z3IndexKeySpace useFullFilter,
// idx/index/z3/Z3IndexKeySpace.scala:240-254): BBOX (inclusive, GeometryProcessing.scala:129)
// AND during (exclusive ms, FastTemporalOperator.scala:123-126) AND the OR over the query
// geometries (GeometryProcessing.process splits a geometry into an OR of parts, :104-136) of
//   INTERSECTS(geom, P)          -> P.intersects(point) = PointLocator.locate != EXTERIOR
//   CONTAINS(P, geom) / WITHIN   -> P.contains(point)   = locate == INTERIOR
// The geometries come as a join index (gm_pip_index): a row that passes the cheap terms costs the
// join's cell lookup (coarse word -> fine word -> list) and, in a boundary cell, one blob walk.  For
// a query-sized index the cell tables and blobs stay in L2, so the scan streams the columns at the
// rate of the strict scan (24 B per row) plus a few L2 hits per candidate row.  Rows are laid out
// as in the other mask kernels (pair_scan: 16-B loads, ballot-interleaved mask words).
enum : int { SP_NONE = 0, SP_INTERSECTS = 1, SP_CONTAINS = 2 };
static_assert(CF_LOG == 3, "k_query_mask packs a fine cell's 3 + 3 bit place in its coarse cell");

template <int OP>
__device__ __forceinline__ bool entry_pred(const PipDev& d, uint32_t e, double px, double py) {
  if ((e >> 30) == CELL_INTERIOR) return true;   // every point of the cell is interior
  const uint32_t ref = e & 0x3fffffffu;
  if (GM_REF_BAD(!blob_ref_ok(d, ref))) { pip_fault(d, PIP_FAULT_BLOB); return false; }
  int loc;
  if (ref & BLOB_COMPACT) {
    int poly;
    loc = compact_locate_lean((const dv2*)(d.compact + 16 * (uint64_t)(ref & (BLOB_COMPACT - 1))), px, py, poly);
  } else {
    const double* b = d.blob + 2 * (uint64_t)ref;
    loc = blob_locate(d, b, *(const int2*)b, px, py);
  }
  return OP == SP_INTERSECTS ? loc != LOC_EXTERIOR : loc == LOC_INTERIOR;
}

// Phases per lane, over the lane's 2 NP rows:
//  1. the streaming terms (16-B loads, registers only); rows inside the index envelope keep their
//     coarse and fine cell numbers;
//  2. the coarse words of all surviving rows (the join's coarse table, coarse_sc: EMPTY / INTERIOR
//     coarse cells and the sub-block masks of mixed ones decide most rows), then the fine words of the
//     rest (cell_sc: the cell words with the boundary shortcuts applied) -- independent loads issued
//     together, so the chain costs two L2 round trips per lane, not two per row;
//  3. the rows still undecided walk one per loop trip, re-reading the row's coordinates (keeping the
//     staged columns live through the walk costs 32 VGPRs): a boundary cell crossed by one or two
//     segments decides from its 32-B line entry (item_locate), only a row near a line or in a cell the
//     shortcuts left walks its blob; a multi-polygon list tests its entries.
// Block shape: FROWS = 4096 rows per block (the shared mask / count / compaction layout) as TPB threads
// x 2 NP rows; 256 x 16 rows by default.  Fewer rows per lane with a geometry term hold fewer VGPRs
// (512 threads: 85 instead of 110) but the wave then waits for its few lookups every 8 rows instead of
// every 16: measured slower (GM_QUERY_TPB, profiles/r5/query_block_shape_ab.txt).
#ifndef GM_QUERY_TPB
#define GM_QUERY_TPB 256   // 256 / 512 / 1024: 2.76 / 4.04 / 5.11 ms per 1B rows (profiles/r5/query_block_shape_ab.txt)
#endif
template <int OP>
struct QueryShape {
  static constexpr int TPB = OP == SP_NONE ? FTPB : GM_QUERY_TPB;
  static constexpr int NP = FROWS / (2 * TPB);
};
template <bool VEC, bool DURING, int OP>
__global__ __launch_bounds__(QueryShape<OP>::TPB) void k_query_mask(const double* __restrict__ x, const double* __restrict__ y,
                                                     const int64_t* __restrict__ t, int64_t n, int has_bbox,
                                                     double bx0, double by0, double bx1, double by1, int64_t lo,
                                                     int64_t hi, PipDev d, uint64_t* __restrict__ mask,
                                                     int32_t* __restrict__ block_counts) {
  constexpr int TPB = QueryShape<OP>::TPB, NP = QueryShape<OP>::NP;
  constexpr int R = 2 * NP;
  const int64_t npairs = n >> 1, nwords = (n + 63) >> 6;
  const int wave = threadIdx.x >> 6;
  const int64_t pbase = (int64_t)blockIdx.x * (TPB * NP);
  dv2 xv[NP], yv[NP];
  lv2 tv[NP];
  uint32_t live = 0;   // bit 2u + j: row j of pair step u exists
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const int64_t p = pbase + (int64_t)u * TPB + threadIdx.x;
    xv[u] = yv[u] = dv2{0.0, 0.0};
    tv[u] = lv2{0, 0};
    if (p < npairs) {
      live |= 3u << (2 * u);
      if (VEC) {
        xv[u] = __builtin_nontemporal_load(&((const dv2*)x)[p]);
        yv[u] = __builtin_nontemporal_load(&((const dv2*)y)[p]);
        if (DURING) tv[u] = __builtin_nontemporal_load(&((const lv2*)t)[p]);
      } else {
        xv[u] = dv2{x[2 * p], x[2 * p + 1]};
        yv[u] = dv2{y[2 * p], y[2 * p + 1]};
        if (DURING) tv[u] = lv2{t[2 * p], t[2 * p + 1]};
      }
    } else if (p == npairs && (n & 1)) {   // the odd last row
      live |= 1u << (2 * u);
      xv[u].x = x[2 * p];
      yv[u].x = y[2 * p];
      if (DURING) tv[u].x = t[2 * p];
    }
  }
  uint32_t pass = 0;
  int fc[R];          // fine cell of each row (geometry term only)
  uint32_t cc[R];     // its coarse cell (low 26 bits) and the fine cell's place in it (top 6 bits)
  static_assert(CF_LOG == 3, "cc packs the fine cell's 3 + 3 bits of position in its coarse cell into bits 26-31");
  constexpr int CF_MASK = (1 << CF_LOG) - 1;
  auto cheap = [&](double px, double py, int64_t tt, int k) {
    bool ok = !has_bbox || (px >= bx0 && px <= bx1 && py >= by0 && py <= by1);
    if (DURING) ok = ok && tt > lo && tt < hi;
    if (OP != SP_NONE) {
      ok = ok && px >= d.gx0 && px <= d.gx1 && py >= d.gy0 && py <= d.gy1;
      const int cx = cell_of(px, d.gx0, d.inv_cw, d.gx), cy = cell_of(py, d.gy0, d.inv_ch, d.gy);
      fc[k] = cy * d.gx + cx;
      // the coarse cell (< 2^20 of them: the grid has at most 2^26 cells) and, in the top 6 bits, the
      // fine cell's place in it (what coarse_mask reads)
      cc[k] = (uint32_t)((cy >> CF_LOG) * d.gxc + (cx >> CF_LOG)) |
              ((uint32_t)((cy & CF_MASK) << CF_LOG | (cx & CF_MASK)) << 26);
    }
    return ok;
  };
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    pass |= (uint32_t)cheap(xv[u].x, yv[u].x, tv[u].x, 2 * u) << (2 * u);
    pass |= (uint32_t)cheap(xv[u].y, yv[u].y, tv[u].y, 2 * u + 1) << (2 * u + 1);
  }
  pass &= live;
  if (OP != SP_NONE && pass) {
    uint32_t cw[R];
#pragma unroll
    for (int k = 0; k < R; ++k) cw[k] = ((pass >> k) & 1u) ? d.coarse_sc[cc[k] & 0x3ffffff] : (CELL_EMPTY << 30);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const uint32_t sb = cc[k] >> 26;
      cw[k] = coarse_mask(cw[k], (int)(sb & 7u), (int)(sb >> 3), d.coarse_fmt);
    }
#pragma unroll
    for (int k = 0; k < R; ++k)
      if ((cw[k] >> 30) == CELL_LIST) cw[k] = d.cell_sc[fc[k]];
    uint32_t slow = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const uint32_t kind = cw[k] >> 30;
      if (kind == CELL_EMPTY) pass &= ~(1u << k);
      else if (kind != CELL_INTERIOR) slow |= 1u << k;   // a blob, or a list of (cell, polygon) entries
    }
    for (; slow; slow &= slow - 1) {
      const int k = __builtin_ctz(slow);
      uint32_t w = cw[0];   // static selects: no register indexing
#pragma unroll
      for (int j = 1; j < R; ++j)
        if (k == j) w = cw[j];
      const int64_t row = 2 * (pbase + (int64_t)(k >> 1) * TPB + threadIdx.x) + (k & 1);
      const double px = x[row], py = y[row];
      bool hit;
      if ((w >> 30) == CELL_LIST) {
        int l0 = 4 * (int)((w & 0x3fffffffu) >> 4), ni = (int)(w & 15u);
        if (GM_REF_BAD((int64_t)l0 + 4 > d.n_list)) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
        else if (ni == LIST_LONG) { ni = (int)d.list_ent[l0]; l0 += 1; }
        if (GM_REF_BAD(ni < 0 || (int64_t)l0 + ni > d.n_list)) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
        hit = false;
        for (int j = 0; j < ni && !hit; ++j) hit = entry_pred<OP>(d, d.list_ent[l0 + j], px, py);
      } else {   // a boundary cell: its line entry (LINE words), else its blob
        int poly;
        const int loc = item_locate<true>(d, w & 0x3fffffffu, px, py, poly);
        hit = OP == SP_INTERSECTS ? loc != LOC_EXTERIOR : loc == LOC_INTERIOR;
      }
      if (!hit) pass &= ~(1u << k);
    }
  }
  int cnt = 0;
#pragma unroll
  for (int u = 0; u < NP; ++u) {
    const uint64_t be = __ballot((pass >> (2 * u)) & 1u), bo = __ballot((pass >> (2 * u + 1)) & 1u);
    cnt += __popcll(be) + __popcll(bo);
    put_pair_words(be, bo, mask, ((pbase + (int64_t)u * TPB + wave * 64) * 2) >> 6, nwords);
  }
  block_count_waves<TPB>(cnt, block_counts);
}
template <bool VEC, bool DURING>
void launch_query(hipStream_t s, unsigned grid, int op, const double* x, const double* y, const int64_t* t, int64_t n,
                  int has_bbox, const double* bb, int64_t lo, int64_t hi, const PipDev& d, uint64_t* mask,
                  int32_t* counts) {
  switch (op) {
    case SP_INTERSECTS:
      hipLaunchKernelGGL((k_query_mask<VEC, DURING, SP_INTERSECTS>), dim3(grid), dim3(QueryShape<SP_INTERSECTS>::TPB), 0, s, x, y, t, n, has_bbox,
                         bb[0], bb[1], bb[2], bb[3], lo, hi, d, mask, counts);
      break;
    case SP_CONTAINS:
      hipLaunchKernelGGL((k_query_mask<VEC, DURING, SP_CONTAINS>), dim3(grid), dim3(QueryShape<SP_CONTAINS>::TPB), 0, s, x, y, t, n, has_bbox,
                         bb[0], bb[1], bb[2], bb[3], lo, hi, d, mask, counts);
      break;
    default:
      hipLaunchKernelGGL((k_query_mask<VEC, DURING, SP_NONE>), dim3(grid), dim3(QueryShape<SP_NONE>::TPB), 0, s, x, y, t, n, has_bbox,
                         bb[0], bb[1], bb[2], bb[3], lo, hi, d, mask, counts);
  }
}

}  // namespace gm

using namespace gm;

extern "C" {

int gm_query_scan(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n, const double* bbox,
                  int has_during, int64_t lo, int64_t hi, const gm_pip_index* geoms, int spatial_op, uint64_t* mask,
                  int64_t* ids, int64_t ids_cap, int64_t* n_match) {
  if (!ctx || n < 0 || ids_cap < 0) return GM_E_INVALID;
  if (spatial_op < GM_SPATIAL_NONE || spatial_op > GM_SPATIAL_CONTAINS) return GM_E_INVALID;
  if (spatial_op != GM_SPATIAL_NONE && !geoms) return GM_E_INVALID;
  if (n == 0) { if (n_match) *n_match = 0; return GM_OK; }
  if (!x || !y || (has_during && !t_ms)) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  ScanBufs b;
  int rc = alloc_scan(ctx, n, mask, 0, b);
  if (rc) return rc;
  const double nobb[4] = {0.0, 0.0, 0.0, 0.0};
  const double* bb = bbox ? bbox : nobb;
  PipDev d = spatial_op != GM_SPATIAL_NONE ? geoms->dev : PipDev{};
  if (spatial_op != GM_SPATIAL_NONE) {   // sticky reference checks
    d.fault = (uint32_t*)(ctx->d_scratch + SCRATCH_FAULT);
    note_fault_call(ctx, FC_QUERY);
  }
  const unsigned grid = (unsigned)((n + FROWS - 1) / FROWS);
  const bool vec = aligned16(x) && aligned16(y) && (!has_during || aligned16(t_ms));
  if (vec) {
    if (has_during) launch_query<true, true>(ctx->stream, grid, spatial_op, x, y, t_ms, n, bbox != nullptr, bb, lo, hi, d, b.mask, b.counts);
    else launch_query<true, false>(ctx->stream, grid, spatial_op, x, y, t_ms, n, bbox != nullptr, bb, lo, hi, d, b.mask, b.counts);
  } else {
    if (has_during) launch_query<false, true>(ctx->stream, grid, spatial_op, x, y, t_ms, n, bbox != nullptr, bb, lo, hi, d, b.mask, b.counts);
    else launch_query<false, false>(ctx->stream, grid, spatial_op, x, y, t_ms, n, bbox != nullptr, bb, lo, hi, d, b.mask, b.counts);
  }
  GM_CHECK_LAUNCH();
  rc = finish_scan(ctx, n, b, ids, ids_cap, n_match);
  free_scan(ctx, mask, b);
  if (rc) return rc;
  if (spatial_op != GM_SPATIAL_NONE && (rc = take_fault(ctx, "gm_query_scan"))) return rc;
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

}  // extern "C"
