// gm_pip_relate.hip -- the row-wise spatial predicate (Spark SQL's st_* UDFs when the join rule does
// not apply): PointLocator's location of point i in polygon poly[i], from the polygon index
// (gm_pip.hpp).  Reference: SpatialRelationFunctions.scala:29-37, SQLFunctionHelper.scala:27-33.
#include <algorithm>
#include <type_traits>

#include "gm_pip.hpp"

namespace gm {

// ------------------------------------------------------------------ row-wise predicate (UDF path)
// st_contains / st_covers / st_intersects / ... evaluated row by row, as Spark SQL runs the UDF when
// the join rule does not apply (SpatialRelationFunctions.scala:29-37 over nullableUDF,
// SQLFunctionHelper.scala:27-33): row i pairs polygon poly[i] with point i.  Every DE-9IM predicate
// of an areal geometry and a point is a function of the point's location in the polygon
// (PointLocator.locate), so the kernel writes that location (LOC_*) and the host maps it.
// The lookup is the join's: cell word chain, then only the entry of polygon poly[i] -- INTERIOR
// decides at once, a blob is walked; no entry means the cell misses the polygon (exterior).
constexpr uint8_t LOC_NULL = 0xff;

__device__ __forceinline__ int entry_locate(const PipDev& d, uint32_t e, double px, double py) {
  if ((e >> 30) == CELL_INTERIOR) return LOC_INTERIOR;
  const uint32_t ref = e & 0x3fffffffu;
  if (GM_REF_BAD(!blob_ref_ok(d, ref))) { pip_fault(d, PIP_FAULT_BLOB); return LOC_EXTERIOR; }
  if (ref & BLOB_COMPACT) {
    int poly;
    return compact_locate((const dv2*)(d.compact + 16 * (uint64_t)(ref & (BLOB_COMPACT - 1))), px, py, poly);
  }
  const double* b = d.blob + 2 * (uint64_t)ref;
  return blob_locate(d, b, *(const int2*)b, px, py);
}

// Per wave: RILP rows per lane per step.  A row resolves at once when its cell is empty, interior, or
// a list without polygon poly[i] (list_poly search); a boundary entry of the row's polygon is queued
// in LDS and the wave walks 64 queued blobs at a time (one per lane), as the join does -- every row
// writes its location exactly once.
#ifndef GM_RILP
#define GM_RILP 2
#endif
constexpr int RILP = GM_RILP;
constexpr int RQCAP = 64 * (RILP + 1);
// VEC: a lane's RILP = 2 rows are adjacent (one 16-B load per coordinate column, one 8-B id load, one
// 2-B location store when both resolve at once); the host picks it when the columns are aligned.
// R32 (rows < 2^32): queue rows as 32-bit values and walk the queue after each of the RILP rows, so
// a queue holds < 128 items (RQCAP32) instead of < 192 and the LDS they free holds the finer coarse
// EMPTY bitmap rm instead of the join's cm
template <bool VEC, bool R32>
__global__ __launch_bounds__(RTPB) void k_pip_relate(const int32_t* __restrict__ poly, const double* __restrict__ px,
                                                     const double* __restrict__ py, int64_t n, int32_t n_polys,
                                                     PipDev d, const int32_t* __restrict__ list_poly,
                                                     uint8_t* __restrict__ loc) {
  static_assert(!VEC || RILP == 2, "adjacent rows per lane are written for RILP = 2");
  constexpr int NW = RTPB / 64;
  constexpr int CAP = R32 ? RQCAP32 : RQCAP;
  constexpr int BM_MAX = R32 ? RM_WORDS_MAX : CM_WORDS_MAX;
  using RowT = typename std::conditional<R32, uint32_t, int64_t>::type;
  __shared__ double s_x[NW][CAP], s_y[NW][CAP];
  __shared__ RowT s_row[NW][CAP];
  __shared__ uint32_t s_e[NW][CAP];
  __shared__ int32_t s_p[NW][CAP];
  // a coarse EMPTY bitmap staged in LDS like k_pip_join_q's: rows in EMPTY coarse blocks skip the
  // coarse gather -- the join's cm (2 x 1 coarse cells per bit at the bench density) or, R32, the
  // finer rm the smaller queues leave room for.  (Round 4's per-polygon core rectangles in LDS beside
  // a bitmap of half the join's resolution answered fewer rows: profiles/r5/relate_bitmap_vs_core_ab.txt)
  __shared__ uint32_t s_cm[BM_MAX];
  const uint32_t* bm = R32 ? d.rm : d.cm;
  const int64_t bm_n = R32 ? d.rm_words : d.cm_words;
  const int bm_sx = R32 ? d.rm_shift : d.cm_shift, bm_sy = R32 ? d.rm_shift_y : d.cm_shift_y;
  const int bm_w = R32 ? d.rm_w : d.cm_w;
  const int64_t cm_words = bm_n <= BM_MAX ? bm_n : 0;
  for (int64_t i = threadIdx.x; i < cm_words; i += RTPB) s_cm[i] = bm[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* qx = s_x[wave]; double* qy = s_y[wave];
  RowT* qr = s_row[wave]; uint32_t* qe = s_e[wave]; int32_t* qp = s_p[wave];
  int qn = 0, qg = 0;   // queued line-entry items (from slot 0 up) and blob items (from CAP - 1 down)
  // walk min(qn, 64) queued items of one kind while the queue holds a full wave, and drain it at the
  // end (< 64 queued before a step's (R32: a row's) <= 64 * RILP (64) new items, so both ends fit CAP;
  // the fuller kind goes first, which leaves < 64 again)
  auto walk = [&](bool drain) {
    while (qn + qg >= 64 || (drain && qn + qg > 0)) {
      wave_lds_sync();
      const bool lines = qn >= qg;
      const int kq = min(lines ? qn : qg, 64);
      const int slot = lines ? qn - kq + lane : CAP - qg + lane;
      if (lane < kq) {
        const uint32_t ref = qe[slot] & 0x3fffffffu;
        const double ex = qx[slot], ey = qy[slot];
        int pl = -1;
        const int l = item_locate(d, ref, ex, ey, pl);
        loc[(int64_t)qr[slot]] = (uint8_t)(pl == qp[slot] ? l : LOC_EXTERIOR);
      }
      wave_lds_sync();
      if (lines) qn -= kq;
      else qg -= kq;
    }
  };
  const int64_t wstep = (int64_t)gridDim.x * NW * (64 * RILP);
  for (int64_t w0 = ((int64_t)blockIdx.x * NW + wave) * (64 * RILP);; w0 += wstep) {
    const bool have = w0 < n;   // uniform per wave
    if (have) {
      int64_t row[RILP];
      int p[RILP];
      double x[RILP], y[RILP];
      uint32_t w[RILP];
      int cx[RILP], cy[RILP];
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        row[u] = VEC ? w0 + RILP * lane + u : w0 + u * 64 + lane;
        p[u] = -1; x[u] = y[u] = 0.0;
      }
      if (VEC && row[1] < n) {
        const uint64_t pp = __builtin_nontemporal_load((const uint64_t*)(poly + row[0]));
        const dv2 a = __builtin_nontemporal_load((const dv2*)(px + row[0]));
        const dv2 b = __builtin_nontemporal_load((const dv2*)(py + row[0]));
        p[0] = (int)(uint32_t)pp; p[1] = (int)(uint32_t)(pp >> 32); x[0] = a.x; x[1] = a.y; y[0] = b.x; y[1] = b.y;
      } else {
#pragma unroll
        for (int u = 0; u < RILP; ++u)
          if (row[u] < n) { p[u] = poly[row[u]]; x[u] = px[row[u]]; y[u] = py[row[u]]; }
      }
      // the rows' coarse gathers are issued together and only then resolved: with the gather and its
      // coarse_mask in one per-row branch the first row's gather was waited for before the second row's
      // was issued
      bool gat[RILP];
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        // the cells of every row, clamped (unused for a row outside the grid): no branch around them
        const bool in = p[u] >= 0 && p[u] < n_polys && x[u] >= d.gx0 && x[u] <= d.gx1 && y[u] >= d.gy0 &&
                        y[u] <= d.gy1;
        cx[u] = cell_of(x[u], d.gx0, d.inv_cw, d.gx);
        cy[u] = cell_of(y[u], d.gy0, d.inv_ch, d.gy);
        bool empty = false;
        if (cm_words) {
          const int b = ((cy[u] >> CF_LOG) >> bm_sy) * bm_w + ((cx[u] >> CF_LOG) >> bm_sx);
          empty = (s_cm[b >> 5] >> (b & 31)) & 1u;
        }
        gat[u] = in && !empty;
      }
      uint32_t craw[RILP];
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        craw[u] = CELL_EMPTY << 30;
        if (gat[u]) craw[u] = d.coarse_sc[(int64_t)(cy[u] >> CF_LOG) * d.gxc + (cx[u] >> CF_LOG)];
      }
#pragma unroll
      for (int u = 0; u < RILP; ++u) w[u] = coarse_mask(craw[u], cx[u], cy[u], d.coarse_fmt);
      // the join's 8-B fine words: a cell crossed by one or two boundary lines carries them inline, so
      // the row decides in registers instead of gathering the 4-B word and then its line entry
      // (10.04-10.16 -> 9.52-9.53 ms per 1B rows, profiles/r5/relate_inline_lines_ab.txt; round 4's
      // attempt, which decided both rows' lines in one pass over more registers, lost)
      uint32_t hi[RILP];
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        hi[u] = 0u;
        if ((w[u] >> 30) == CELL_LIST) {
          const uint2 w8 = d.cell_sc8[(int64_t)cy[u] * d.gx + cx[u]];
          w[u] = w8.x; hi[u] = w8.y;
        }
      }
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        if (sc8_inline(make_uint2(w[u], hi[u]))) {
          const uint2 w8 = make_uint2(w[u], hi[u]);
          const int l = sc8_locate(w8, x[u], y[u], d, cx[u], cy[u]);
          if (l == LOC_INTERIOR) w[u] = (CELL_INTERIOR << 30) | (uint32_t)sc8_poly(w8);   // compared with p below
          else if (l == LOC_EXTERIOR) w[u] = CELL_EMPTY << 30;
          else w[u] = d.cell_sc[(int64_t)cy[u] * d.gx + cx[u]];   // near a line: the entry, then the blob
        }
      }
      uint8_t rv[RILP];
      bool dir[RILP];
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        uint8_t r = LOC_EXTERIOR;
        bool queue = false;
        uint32_t e = w[u];
        const uint32_t kind = e >> 30;
        if (p[u] < 0 || p[u] >= n_polys) {
          r = LOC_NULL;
        } else if (kind == CELL_INTERIOR) {
          r = (int)(e & 0x3fffffffu) == p[u] ? LOC_INTERIOR : LOC_EXTERIOR;
        } else if (kind == CELL_BOUNDARY) {
          queue = true;   // the blob's polygon is checked when it is walked
        } else if (kind == CELL_LIST) {
          int l0 = 4 * (int)((e & 0x3fffffffu) >> 4), ni = (int)(e & 15u);
          bool found = false;
          if (GM_REF_BAD((int64_t)l0 + 4 > d.n_list)) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
          else if (ni <= 4) {
            // a short list is one 16-B group (lists start at multiples of 4 slots): its polygon ids
            // and entries in two independent loads instead of a serial search
            const int4 lp = *(const int4*)(list_poly + l0);
            const uint4 le = *(const uint4*)(d.list_ent + l0);
            const int pv = p[u];
            found = true;
            if (ni > 0 && lp.x == pv) e = le.x;
            else if (ni > 1 && lp.y == pv) e = le.y;
            else if (ni > 2 && lp.z == pv) e = le.z;
            else if (ni > 3 && lp.w == pv) e = le.w;
            else found = false;
            ni = 0;
          } else if (ni == LIST_LONG) { ni = (int)d.list_ent[l0]; l0 += 1; }
          if (GM_REF_BAD(ni < 0 || (int64_t)l0 + ni > d.n_list)) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
          int j = 0;
          while (j < ni && list_poly[l0 + j] != p[u]) ++j;
          if (j < ni) { e = d.list_ent[l0 + j]; found = true; }
          if (found) {
            if ((e >> 30) == CELL_INTERIOR) r = LOC_INTERIOR;
            else queue = true;
          }
        }
        rv[u] = r;
        dir[u] = row[u] < n && !queue;
        if (!VEC && dir[u]) loc[row[u]] = r;
        // line-entry items and blob items on separate ends, so an evaluation round runs one kind
        const bool ln = (e & (BLOB_COMPACT | SC_LINE)) == (BLOB_COMPACT | SC_LINE) && d.line_ent;
        const bool qv = queue && row[u] < n;
        const uint64_t ml = __ballot(qv && ln), mb = __ballot(qv && !ln);
        if (qv) {
          const int o = ln ? qn + lanes_below(ml) : CAP - 1 - qg - lanes_below(mb);
          qx[o] = x[u]; qy[o] = y[u]; qr[o] = (RowT)row[u]; qe[o] = e; qp[o] = p[u];
        }
        qn += __popcll(ml);
        qg += __popcll(mb);
        if (R32) walk(false);
      }
      if (VEC) {
        if (dir[0] && dir[1]) *(uint16_t*)(loc + row[0]) = (uint16_t)(rv[0] | (rv[1] << 8));
        else {
          if (dir[0]) loc[row[0]] = rv[0];
          if (dir[1]) loc[row[1]] = rv[1];
        }
      }
    }
    walk(!have);
    if (!have) break;
  }
}

}  // namespace gm

using namespace gm;

extern "C" {

int gm_pip_relate(gm_ctx* ctx, const gm_pip_index* ix, const int32_t* poly, const double* px, const double* py,
                  int64_t n, uint8_t* loc) {
  if (!ctx || !ix || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!poly || !px || !py || !loc) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  PipDev dv = ix->dev;
  dv.fault = (uint32_t*)(ctx->d_scratch + SCRATCH_FAULT);   // sticky reference checks, as the join's
  note_fault_call(ctx, FC_RELATE);
  const bool vec = RILP == 2 && ((uintptr_t)px | (uintptr_t)py) % 16 == 0 && (uintptr_t)poly % 8 == 0 &&
                   (uintptr_t)loc % 2 == 0;
  // 32-bit queue rows and the finer bitmap when the rows fit and the index built it
  const bool r32 = !ctx->relate_rows64 && n <= (int64_t)UINT32_MAX && dv.rm_words > 0 && dv.rm_words <= RM_WORDS_MAX;
  auto* kern = vec ? (r32 ? k_pip_relate<RILP == 2, true> : k_pip_relate<RILP == 2, false>)
                   : (r32 ? k_pip_relate<false, true> : k_pip_relate<false, false>);
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(resident_blocks((const void*)kern, ctx->device, RTPB, 1),
                                                                          (n + RTPB * RILP - 1) / (RTPB * RILP)));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(RTPB), 0, ctx->stream, poly, px, py, n, ix->n_polys, dv, ix->list_poly, loc);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

}  // extern "C"
