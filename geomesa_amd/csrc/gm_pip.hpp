// gm_pip.hpp -- the point-in-polygon index shared by the join (gm_pip_join.hip), the row-wise
// predicate (gm_pip_relate.hip), the fused query scan (gm_pip_query.hip) and the index build
// (gm_pip_build.hip): its device view (PipDev), the cell-word encoding, and the exact locators a
// kernel runs on a (cell, polygon) pair -- JTS 1.20 semantics throughout.
//
// Reference path: ST_Contains = geom1.contains(geom2) (geomesa-spark-jts/.../udf/SpatialRelationFunctions.scala:29)
// evaluated per candidate pair by GeoMesaJoinRelation.sweeplineJoin / OverlapAction
// (geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91, OverlapAction.scala:25-41) after grid
// partitioning (RelationUtils.scala:30-157).  JTS Geometry.contains(point): envelope covers, then
// relate -> PointLocator with the Mod-2 boundary rule; rings via RayCrossingCounter with the robust
// CGAlgorithmsDD orientation (filter + double-double).  Boundary points are NOT contained.
//
// Index (built once per polygon set -- the analogue of broadcasting the polygon side of the join):
//   * a uniform grid over the polygon set's envelope.  Every (cell, polygon) pair whose envelopes
//     meet is INTERIOR (no segment of the polygon meets the inflated cell and the cell is inside:
//     every point of the cell is contained, no arithmetic at all), EXTERIOR (dropped) or BOUNDARY;
//   * a BOUNDARY pair carries one record per ring of the polygon: the ring segments that meet the
//     inflated cell (tested exactly with RayCrossingCounter.countSegment), plus the crossing parity
//     of all segments to the RIGHT of the cell as a function of the point's y.  Within the cell's
//     y-band a segment that misses the inflated cell lies wholly left (never counted) or wholly
//     right (counted iff it straddles y: ymin <= y < ymax, the half-open rule of countSegment), so
//     that parity is piecewise constant with breakpoints at segment end-point y values; it is
//     precomputed per interval (<= 63 breakpoints, else the record falls back to the slab walk).
//     Geometric and JTS answers agree there: those segments are at least one cell away from the
//     point, where the orientation filter is exact.
//   * per ring y-slab buckets of all segments: the fallback walk (every segment whose y-range holds
//     the point's y -- the only ones countSegment can count).
// A point costs one cell lookup plus, in a boundary cell, ~2 exact segment tests.
#pragma once

#include <math.h>
#include <stdio.h>

#include <vector>

#include "gm_internal.hpp"

namespace gm {

enum : int { LOC_EXTERIOR = 0, LOC_BOUNDARY = 1, LOC_INTERIOR = 2 };

struct RingDev {
  double minx, miny, maxx, maxy;  // ring envelope (empty ring: +inf/-inf)
  double y0, inv_h;               // slab(y) = clamp(floor((y - y0) * inv_h), 0, ns - 1)
  int32_t ns, slab_base;          // slab_off[slab_base .. slab_base + ns]
};

struct Edge {
  double p1x, p1y, p2x, p2y;  // countSegment(p1 = ring[i], p2 = ring[i-1])
};

struct PipDev {
  const RingDev* rings;          // fallback slab walk
  const int32_t* slab_off;
  const Edge* slab_edges;
  const uint32_t* coarse_word;   // per coarse cell (CF x CF fine cells): EMPTY, INTERIOR or LIST = "look at the fine word"
  const uint32_t* cell_word;     // per cell: kind << 30 | payload (see CELL_*)
  const double* compact;         // compact blobs: 16 words (one 128-B line) each
  const uint32_t* list_ent;      // entries in cell-word form (kind INTERIOR or BOUNDARY)
  const double* blob;            // boundary blobs, 16-byte aligned
  const uint32_t* cell_sc;       // per cell: the cell word with the boundary shortcuts applied (k_build_shortcut)
  const uint32_t* coarse_sc;     // the join's coarse words over cell_sc; LIST words carry sub-block masks
  int32_t coarse_fmt;            // COARSE_EMPTY_MASK / COARSE_MAIN (see coarse_mask)
  const uint4* line_ent;         // line shortcuts, two uint4 each (see "Boundary shortcuts")
  const uint2* cell_sc8;         // the join's 8-B fine words: cell_sc, with one-line LINE words inline (sc8_*)
  double gx0, gy0, gx1, gy1, inv_cw, inv_ch;
  int32_t gx, gy, gxc;
  int32_t op;                    // join predicate: JOIN_CONTAINS (interior) or JOIN_INTERSECTS (not exterior)
  // reference checks: every blob / line / list reference a kernel follows is bounded by these sizes
  // (make_shortcut); a reference beyond them sets a PIP_FAULT_* bit in *fault (the call's scratch
  // word, null = not checked by this caller) and is treated as EXTERIOR, never dereferenced
  uint32_t* fault;
  int64_t n_line, n_compact_lines, n_blob16, n_list;
  // coarse EMPTY bitmap (make_shortcut; staged in LDS by the direct join): bit (by * cm_w + bx) set when
  // every coarse cell of block (bx, by) = coarse cells [bx << cm_shift, (bx + 1) << cm_shift) x
  // [by << cm_shift_y, (by + 1) << cm_shift_y) is EMPTY; cm_words = 0: no bitmap
  const uint32_t* cm;
  int32_t cm_shift, cm_shift_y, cm_w;
  int64_t cm_words;
  // the same bitmap at the row predicate's resolution (RM_WORDS_MAX: what its 32-bit-row queues leave)
  const uint32_t* rm;
  int32_t rm_shift, rm_shift_y, rm_w;
  int64_t rm_words;
};

enum : uint32_t { PIP_FAULT_LINE = 1, PIP_FAULT_COMPACT = 2, PIP_FAULT_BLOB = 4, PIP_FAULT_LIST = 8, PIP_FAULT_QUEUE = 16 };

__device__ __forceinline__ void pip_fault(const PipDev& d, uint32_t code) {
  if (d.fault) atomicOr(d.fault, code);
}
// a reference / queue check; GM_NO_REF_CHECKS (timing variant only) compiles every check out to price
// them.  The shipped library (GM_PRODUCT_BUILD, geomesa_amd/build.py) refuses it at compile time too, so
// no build path can ship without the device reference checks.
#if defined(GM_PRODUCT_BUILD) && defined(GM_NO_REF_CHECKS)
#error "GM_NO_REF_CHECKS is a timing variant: it cannot be built into the shipped library"
#endif
#ifdef GM_NO_REF_CHECKS
#define GM_REF_BAD(c) (false)
#else
#define GM_REF_BAD(c) (c)
#endif


#ifndef GM_CF_LOG
#define GM_CF_LOG 3
#endif
#ifndef GM_MAX_CELLS_LOG
#define GM_MAX_CELLS_LOG 26
#endif
constexpr int CF_LOG = GM_CF_LOG;   // coarse cell = 8 x 8 fine cells: the coarse table (<= 4 MB) stays L2-resident

// cell word kinds (2 high bits; 30-bit payload)
enum : uint32_t { CELL_INTERIOR = 0, CELL_BOUNDARY = 1, CELL_LIST = 2, CELL_EMPTY = 3 };
// BOUNDARY payload: bit 29 set = compact blob index, else generic blob offset (16-B units)
constexpr uint32_t BLOB_COMPACT = 1u << 29;
// LIST payload: list_ent offset << 4 | count; count 15 = long list whose count is list_ent[offset]
constexpr int LIST_LONG = 15;

// is the blob reference of a BOUNDARY entry (payload `ref`, LINE words excluded) inside the index?
__device__ __forceinline__ bool blob_ref_ok(const PipDev& d, uint32_t ref) {
  if (ref & BLOB_COMPACT) return (uint64_t)(ref & (BLOB_COMPACT - 1)) < (uint64_t)d.n_compact_lines;
  return (uint64_t)ref < (uint64_t)d.n_blob16;
}

// Compact blob (single-ring polygon, 4 * segments + breakpoints <= 30 in the cell): one or two
// 128-B lines of 16 words in `compact`, addressed by line index.
//   w0: int32 polygon | int32 meta (segments | lines << 8), w1: parity bits,
//   segment j (p1x p1y p2x p2y) at words CSEG[j] = 2, 6, 10 (line 0), 16, 20, 24, 28 (line 1);
//   every other word of the record is a breakpoint slot (+inf when unused).
// The breakpoint count k = #(slots <= y) does not depend on slot order, so the record is evaluated
// with static indexing, line by line: crossings = parity bit k + segment crossings, exactly the
// RayCrossingCounter walk of a generic one-ring blob.
constexpr int CSEG_MAX = 7;
__host__ __device__ constexpr int cseg_word(int j) { return j < 3 ? 2 + 4 * j : 16 + 4 * (j - 3); }

struct RingHdr {
  int16_t n_edge, n_brk, flags, pad;
};

// the cell of v on a g-cell axis, clamped (NaN -> 0).  Branch-free: a clamp by maxNum / minNum (NaN -> 0)
// instead of two early returns, which compiled to exec-mask branches in every stream step
__device__ __forceinline__ int cell_of(double v, double v0, double inv, int g) {
  const double c = floor(__dmul_rn(__dsub_rn(v, v0), inv));
  return (int)__builtin_fmin(__builtin_fmax(c, 0.0), (double)(g - 1));
}

// RayCrossingCounter.countSegment (JTS 1.20); returns true when the point is on the segment
__device__ __forceinline__ bool count_segment(double p1x, double p1y, double p2x, double p2y, double px, double py,
                                              int& crossings) {
  if (p1x < px && p2x < px) return false;
  if (px == p2x && py == p2y) return true;
  if (p1y == py && p2y == py) {
    double mn = p1x, mx = p2x;
    if (mn > mx) { mn = p2x; mx = p1x; }
    return px >= mn && px <= mx;
  }
  if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
    int orient = jts_orientation(p1x, p1y, p2x, p2y, px, py);
    if (orient == 0) return true;
    if (p2y < p1y) orient = -orient;
    if (orient == 1) crossings++;
  }
  return false;
}

// fallback: RayCrossingCounter.locatePointInRing over the point's y-slab
// (takes the three arrays by value: a reference to the kernel's PipDev argument would force the
// whole struct into scratch and put scratch loads in front of every index lookup)
static __device__ __noinline__ int locate_ring_slab(const RingDev* __restrict__ rings, const int32_t* __restrict__ slab_off,
                                             const Edge* __restrict__ slab_edges, int r, double px, double py) {
  const RingDev rd = rings[r];
  if (!(px >= rd.minx && px <= rd.maxx && py >= rd.miny && py <= rd.maxy)) return LOC_EXTERIOR;
  const int s = cell_of(py, rd.y0, rd.inv_h, rd.ns);
  const int e0 = slab_off[rd.slab_base + s], e1 = slab_off[rd.slab_base + s + 1];
  int crossings = 0;
  for (int e = e0; e < e1; ++e) {
    const Edge g = slab_edges[e];
    if (count_segment(g.p1x, g.p1y, g.p2x, g.p2y, px, py, crossings)) return LOC_BOUNDARY;
  }
  return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

// PointLocator.locate(point) for a BOUNDARY pair from its blob: the polygon's parts
// (locateInPolygon: shell, then holes) with the Mod-2 rule across parts
__device__ inline int blob_locate(const PipDev& d, const double* b, int2 h, double px, double py) {
  const double* w = b + 1;
  bool is_in = false, skip = true, started = false;
  int nb = 0, cur = LOC_EXTERIOR;
  for (int r = 0; r < h.y; ++r) {
    const RingHdr rh = *(const RingHdr*)w;
    const uint64_t parity = *(const uint64_t*)(w + 1);
    const double* eg = w + 2;
    const double* bk = eg + 4 * rh.n_edge;
    w = bk + rh.n_brk;
    if (rh.flags & 1) {  // a new part: settle the previous one
      if (started) { if (cur == LOC_INTERIOR) is_in = true; if (cur == LOC_BOUNDARY) nb++; }
      started = true;
      skip = false;
    } else if (skip) {
      continue;
    }
    int loc;
    if (rh.flags & 2) {
      loc = locate_ring_slab(d.rings, d.slab_off, d.slab_edges, (int)(uint32_t)parity, px, py);
    } else {
      int k = 0;
      for (int j = 0; j < rh.n_brk; ++j) k += bk[j] <= py;
      int crossings = (int)((parity >> k) & 1ull);
      loc = -1;
      for (int j = 0; j < rh.n_edge; ++j)
        if (count_segment(eg[4 * j], eg[4 * j + 1], eg[4 * j + 2], eg[4 * j + 3], px, py, crossings)) {
          loc = LOC_BOUNDARY;
          break;
        }
      if (loc < 0) loc = (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
    }
    if (rh.flags & 1) {          // shell
      cur = loc;
      skip = loc != LOC_INTERIOR;
    } else {                     // hole of a part whose shell holds the point
      if (loc == LOC_INTERIOR) { cur = LOC_EXTERIOR; skip = true; }
      else if (loc == LOC_BOUNDARY) { cur = LOC_BOUNDARY; skip = true; }
    }
  }
  if (started) { if (cur == LOC_INTERIOR) is_in = true; if (cur == LOC_BOUNDARY) nb++; }
  if (nb & 1) return LOC_BOUNDARY;
  return (nb > 0 || is_in) ? LOC_INTERIOR : LOC_EXTERIOR;
}

enum : int32_t { JOIN_CONTAINS = 0, JOIN_INTERSECTS = 1 };
// the join predicate on a located point: Geometry.contains (INTERIOR) or intersects / covers (not EXTERIOR)
__device__ __forceinline__ bool join_hit(int32_t op, int loc) {
  return op == JOIN_INTERSECTS ? loc != LOC_EXTERIOR : loc == LOC_INTERIOR;
}

// Geometry.contains(point): INTERIOR only (a point on the boundary is not contained)
__device__ __forceinline__ bool blob_contains(const PipDev& d, const double* b, int2 h, double px, double py) {
  return blob_locate(d, b, h, px, py) == LOC_INTERIOR;
}

// one line (16 words, 8 independent 16-B loads) of a compact blob: breakpoint count and segments
template <int LINE>
__device__ __forceinline__ void compact_line(const dv2* __restrict__ c, int E, double px, double py, int& k,
                                             int& cr, bool& on) {
  dv2 q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = c[8 * LINE + i];
  auto word = [&](int w) -> double { return (w & 1) ? q[(w & 15) >> 1].y : q[(w & 15) >> 1].x; };
#pragma unroll
  for (int w = 16 * LINE; w < 16 * LINE + 16; ++w) {
    if (w < 2) continue;
    int seg = -1;   // segment group holding word w (compile-time)
#pragma unroll
    for (int j = 0; j < CSEG_MAX; ++j)
      if (w >= cseg_word(j) && w < cseg_word(j) + 4) seg = j;
    if (seg < 0 || seg >= E) k += word(w) <= py;     // a breakpoint slot (+inf when unused)
  }
#pragma unroll
  for (int j = 0; j < CSEG_MAX; ++j) {
    if (cseg_word(j) / 16 != LINE) continue;
    const int w0 = cseg_word(j);
    if (j < E && !on) on = count_segment(word(w0), word(w0 + 1), word(w0 + 2), word(w0 + 3), px, py, cr);
  }
}

__device__ __forceinline__ int compact_locate(const dv2* __restrict__ c, double px, double py, int& poly) {
  const dv2 h = c[0];
  const int64_t meta = __double_as_longlong(h.x);
  poly = (int)meta;
  const int E = (int)((meta >> 32) & 0xff), lines = (int)((meta >> 40) & 0xff);
  int k = 0, cr = 0;
  bool on = false;
  compact_line<0>(c, E, px, py, k, cr, on);
  if (lines > 1) compact_line<1>(c, E, px, py, k, cr, on);
  if (on) return LOC_BOUNDARY;
  cr += (int)(((uint64_t)__double_as_longlong(h.y) >> k) & 1ull);
  return (cr & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

// compact_locate with one 16-B load at a time (a rolled loop over the record's 2 x 8 pairs of words):
// the same arithmetic in the same order per segment and the same breakpoint count, for kernels whose
// walk must not hold the two lines' 64 VGPRs (the fused query scan's block-level walk).  Segment j
// occupies the word pairs cseg_word(j) / 2 and cseg_word(j) / 2 + 1; every other pair is two
// breakpoint slots (a segment slot past E included).
__device__ inline int compact_locate_lean(const dv2* __restrict__ c, double px, double py, int& poly) {
  const dv2 h = c[0];
  const int64_t meta = __double_as_longlong(h.x);
  poly = (int)meta;
  const int E = (int)((meta >> 32) & 0xff), lines = (int)((meta >> 40) & 0xff);
  int k = 0, cr = 0;
  bool on = false;
  const int np = lines > 1 ? 16 : 8;
  for (int i = 1; i < np; ++i) {
    // segment j starting at pair i: i = 1, 3, 5 (line 0), 8, 10, 12, 14 (line 1)
    const int j = (i < 7 && (i & 1)) ? (i - 1) / 2 : ((i >= 8 && !(i & 1)) ? 3 + (i - 8) / 2 : -1);
    if (j >= 0 && j < E) {
      const dv2 a = c[i], b = c[i + 1];
      if (!on) on = count_segment(a.x, a.y, b.x, b.y, px, py, cr);
      ++i;   // the segment's second pair
    } else {
      const dv2 q = c[i];
      k += (q.x <= py) + (q.y <= py);
    }
  }
  if (on) return LOC_BOUNDARY;
  cr += (int)(((uint64_t)__double_as_longlong(h.y) >> k) & 1ull);
  return (cr & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

__device__ __forceinline__ bool compact_contains(const dv2* __restrict__ c, double px, double py, int& poly) {
  return compact_locate(c, px, py, poly) == LOC_INTERIOR;
}

// Boundary shortcuts.  A BOUNDARY (cell, polygon) word stands for every ring segment whose bounding
// box meets the cell; the segments that actually cross the cell are found once, on the device
// (k_build_shortcut), and the join walks cell_sc, a copy of the cell words where
//  * a cell crossed by none of them has one location (no boundary inside it): its word becomes
//    INTERIOR(polygon) or EMPTY;
//  * a cell crossed by one or two segments gets a LINE word and a line entry: the segments' lines in
//    cell units, f(u, v) = A u + B v - C (int16 A, B with max |A|, |B| = 2^14, int24 C, |f - f_exact| <=
//    SC_DEV over the cell), and a location for each combination of sides.  Each combination of
//    open half-planes meets the (convex) cell in a convex region that no boundary crosses, so the
//    location is constant there; it is found by locating test points of that region from the blob.
//    A point at least SC_T from every line takes its region's location; a point nearer a line (and
//    so every boundary point) or in a region without a test point takes the exact blob walk from
//    the entry's original word.
// Every location comes from the blob's own PointLocator walk, so results are those of the blob.
// Entry = two uint4: {cell word, polygon, A1 | B1 << 16, C1 | region flags << 24},
// {A2 | B2 << 16, C2 | lines << 24, 0, 0}; region r = side1 + 2 side2 (side 0: f > 0) has flag bits
// 2r (located) and 2r + 1 (interior).
constexpr double SC_DEV = 4.0;   // quantization deviation allowed over the cell (units of 2^-14 cell)
constexpr double SC_T = 6.0;     // decision threshold: SC_DEV plus ample room for FP64 rounding
// LINE words: BOUNDARY | BLOB_COMPACT | SC_LINE | entry (compact blob indices stay below SC_LINE)
constexpr uint32_t SC_LINE = 1u << 28;

// f(u, v) of a point on one quantized line (ab = A | B << 16, c = C in the low 24 bits), with u, v
// its position in cell units inside cell (cx, cy) (cell_of's arithmetic)
__device__ __forceinline__ double shortcut_f(uint32_t ab, uint32_t c, double x, double y, const PipDev& d, int cx, int cy) {
  const double u = __dsub_rn(__dmul_rn(__dsub_rn(x, d.gx0), d.inv_cw), (double)cx);
  const double v = __dsub_rn(__dmul_rn(__dsub_rn(y, d.gy0), d.inv_ch), (double)cy);
  const double A = (double)(int16_t)(ab & 0xffffu), B = (double)(int16_t)(ab >> 16);
  const double C = (double)((int32_t)(c << 8) >> 8);
  return __dsub_rn(__dadd_rn(__dmul_rn(A, u), __dmul_rn(B, v)), C);
}

// the region of a point (side bits), or -1 within SC_T of a line
__device__ __forceinline__ int line_region(const uint4 e0, const uint4 e1, double x, double y, const PipDev& d, int cx,
                                           int cy, double t) {
  const double g1 = shortcut_f(e0.z, e0.w, x, y, d, cx, cy);
  if (!(g1 > t || g1 < -t)) return -1;
  int r = g1 > t ? 0 : 1;
  if ((e1.y >> 24) > 1) {
    const double g2 = shortcut_f(e1.x, e1.y, x, y, d, cx, cy);
    if (!(g2 > t || g2 < -t)) return -1;
    r |= g2 > t ? 0 : 2;
  }
  return r;
}

// a point's location from a line entry: LOC_INTERIOR / LOC_EXTERIOR, or -1 (the blob decides)
__device__ __forceinline__ int line_locate(const uint4 e0, const uint4 e1, double x, double y, const PipDev& d) {
  const int r = line_region(e0, e1, x, y, d, cell_of(x, d.gx0, d.inv_cw, d.gx), cell_of(y, d.gy0, d.inv_ch, d.gy), SC_T);
  if (r < 0) return -1;
  const uint32_t fl = e0.w >> 24;
  if (!((fl >> (2 * r)) & 1u)) return -1;
  return ((fl >> (2 * r + 1)) & 1u) ? LOC_INTERIOR : LOC_EXTERIOR;
}

// The join's 8-B fine words (cell_sc8, derived from cell_sc and line_ent by make_shortcut).  A
// beyond-L2 gather costs the same for 4 or 16 B per lane (tools/gather_probe.hip: 56-59 G/s either
// way), so a LINE cell carries its lines in its fine word when they fit, and its points decide with
// one gather instead of two (fine word, then the 32-B entry):
//   tag (bits 63-62) 0: the low half is the cell_sc word (high half 0);
//   tag 1, one line: bits 61-48 polygon (< 2^14), 47-44 region flags as in the entry (2r located,
//          2r + 1 interior; r = 0 where f > 0), 43-30 A, 29-16 B (int14), 15-0 C (int16):
//          f(u, v) = A u + B v - C in units of 2^-12 cell, the entry's line requantized (A / 4 ...).
//          The entry's line is within SC_DEV / 4 = 1 unit of the exact line over the cell and the
//          requantization adds <= 1.52, so a point with |f| > SC8_T is on the exact line's side
//          sign(f) and takes that region's location;
//   tag 2, two lines meeting inside the cell (the two segments of a vertex in the cell): bits 61-48
//          polygon, 47-40 the entry's flags of regions r = side1 + 2 side2, 39-30 / 29-20 the lines'
//          intersection V = ((a + 0.5) / 1024, (b + 0.5) / 1024) in cell units, 19-10 / 9-0 each line's
//          normal direction (A, B) as an angle q 2 pi / 1024.  f_k = cos(q_k) (u - Vu) + sin(q_k) (v - Vv)
//          is within SC8_T2 of the signed distance (cells) to the exact line k over the cell: the
//          entry's lines are within 4 / 2^14, V within 0.5 sqrt(2) / 1024, the angle within pi / 1024 at
//          most sqrt(2) from V, plus float rounding.
// A nearer point takes the original word's blob (cell_word), as the entry's near-line points do.
constexpr double SC8_T = 4.0;
constexpr float SC8_T2 = 7.0e-3f;
__device__ __forceinline__ bool sc8_inline(uint2 w) { return (w.y >> 30) == 1u || (w.y >> 30) == 2u; }
__device__ __forceinline__ int sc8_poly(uint2 w) { return (int)((w.y >> 16) & 0x3fffu); }
// (sin, cos) of the angle q 2 pi / 1024: quadrant q >> 8, then Taylor series in float of the angle within
// the quadrant (< pi / 2: remainders below 4e-6, far inside SC8_T2's margin)
__device__ __forceinline__ void sc8_dir(uint32_t q, float& sn, float& cs) {
  const float a = (float)(q & 255u) * (6.2831853071795865f / 1024.0f), a2 = a * a;
  const float s0 = a * (1.0f - a2 * (1.0f / 6.0f - a2 * (1.0f / 120.0f - a2 * (1.0f / 5040.0f - a2 * (1.0f / 362880.0f)))));
  const float c0 = 1.0f - a2 * (0.5f - a2 * (1.0f / 24.0f - a2 * (1.0f / 720.0f - a2 * (1.0f / 40320.0f - a2 * (1.0f / 3628800.0f)))));
  switch (q >> 8) {
    case 0: sn = s0; cs = c0; break;
    case 1: sn = c0; cs = -s0; break;
    case 2: sn = -s0; cs = -c0; break;
    default: sn = -c0; cs = s0; break;
  }
}

// LOC_INTERIOR / LOC_EXTERIOR from an inline word, or -1 (near a line, or an unlocated region)
__device__ __forceinline__ int sc8_locate(uint2 w, double x, double y, const PipDev& d, int cx, int cy) {
  const uint64_t v = ((uint64_t)w.y << 32) | w.x;
  const double u = __dsub_rn(__dmul_rn(__dsub_rn(x, d.gx0), d.inv_cw), (double)cx);
  const double t = __dsub_rn(__dmul_rn(__dsub_rn(y, d.gy0), d.inv_ch), (double)cy);
  uint32_t fl, r;
  if ((w.y >> 30) == 1u) {
    const double A = (double)((int64_t)(v << 20) >> 50), B = (double)((int64_t)(v << 34) >> 50);
    const double C = (double)((int64_t)(v << 48) >> 48);
    const double f = __dsub_rn(__dadd_rn(__dmul_rn(A, u), __dmul_rn(B, t)), C);
    if (!(f > SC8_T || f < -SC8_T)) return -1;
    fl = (uint32_t)(v >> 44) & 15u;
    r = f > SC8_T ? 0u : 1u;
  } else {
    const float du = (float)(u - ((double)((v >> 30) & 1023u) + 0.5) * (1.0 / 1024.0));
    const float dv = (float)(t - ((double)((v >> 20) & 1023u) + 0.5) * (1.0 / 1024.0));
    float s1, c1, s2, c2;
    sc8_dir((uint32_t)(v >> 10) & 1023u, s1, c1);
    sc8_dir((uint32_t)v & 1023u, s2, c2);
    const float f1 = c1 * du + s1 * dv, f2 = c2 * du + s2 * dv;
    if (!(f1 > SC8_T2 || f1 < -SC8_T2) || !(f2 > SC8_T2 || f2 < -SC8_T2)) return -1;
    fl = (uint32_t)(v >> 40) & 255u;
    r = (f1 > 0.0f ? 0u : 1u) + (f2 > 0.0f ? 0u : 2u);
  }
  if (!((fl >> (2 * r)) & 1u)) return -1;
  return ((fl >> (2 * r + 1)) & 1u) ? LOC_INTERIOR : LOC_EXTERIOR;
}

// The join's coarse table (coarse_sc, 4 B per coarse cell like coarse_word, so it stays L2-resident)
// is built over cell_sc: EMPTY / INTERIOR(p) when all its fine cells carry that word, else LIST with
// bit s of the payload set when all fine cells of sub-block s (4 x 4 sub-blocks of 2 x 2 fine
// cells) are EMPTY: a point there needs no fine lookup.
// With fewer than 2^14 polygons (COARSE_MAIN) the payload instead holds 8 sub-blocks of 4 x 2 fine
// cells with an EMPTY bit and an INTERIOR-of-"main" bit each, main being the polygon of the coarse
// cell's first INTERIOR fine cell (14 bits): 13.46 -> 13.27 ms on the counties.
constexpr int SUB_LOG = CF_LOG - 2;
static_assert(CF_LOG >= 2, "sub-block masks need at least 4 x 4 fine cells per coarse cell");
enum : int32_t { COARSE_EMPTY_MASK = 0, COARSE_MAIN = 1 };

__device__ __forceinline__ uint32_t coarse_mask(uint32_t w, int cx, int cy, int32_t fmt) {
  if ((w >> 30) != CELL_LIST) return w;
  constexpr int CM = (1 << CF_LOG) - 1;
  if (fmt == COARSE_MAIN) {   // 8 sub-blocks of 4 x 2: EMPTY mask | INTERIOR(main) mask << 8 | main << 16
    const int sub = (((cy & CM) >> (CF_LOG - 2)) << 1) | ((cx & CM) >> (CF_LOG - 1));
    if ((w >> sub) & 1u) return CELL_EMPTY << 30;
    if ((w >> (8 + sub)) & 1u) return (CELL_INTERIOR << 30) | ((w >> 16) & 0x3fffu);
    return w;
  }
  const int sub = (((cy & CM) >> SUB_LOG) << 2) | ((cx & CM) >> SUB_LOG);   // 16 sub-blocks of 2 x 2: EMPTY mask
  return ((w >> sub) & 1u) ? (CELL_EMPTY << 30) : w;
}

// PointLocator's location of a point for one BOUNDARY item (ref = the word's payload): a line
// shortcut (near the line: the entry's own blob), a compact blob or a generic blob.  LEAN: the compact
// blob one 16-B load at a time (compact_locate_lean)
template <bool LEAN = false>
__device__ __forceinline__ int item_locate(const PipDev& d, uint32_t ref, double x, double y, int& poly) {
  int loc = -1;
  if ((ref & BLOB_COMPACT) && d.line_ent && (ref & SC_LINE)) {
    const uint64_t li = ref & (SC_LINE - 1);
    if (GM_REF_BAD(li >= (uint64_t)d.n_line)) { pip_fault(d, PIP_FAULT_LINE); poly = -1; return LOC_EXTERIOR; }
    const uint4 e0 = d.line_ent[2 * li], e1 = d.line_ent[2 * li + 1];
    poly = (int)e0.y;
    loc = line_locate(e0, e1, x, y, d);
    ref = e0.x & 0x3fffffffu;
  }
  if (loc >= 0) return loc;
  if (ref & BLOB_COMPACT) {
    const uint64_t ci = ref & (BLOB_COMPACT - 1);
    if (GM_REF_BAD(ci >= (uint64_t)d.n_compact_lines)) { pip_fault(d, PIP_FAULT_COMPACT); poly = -1; return LOC_EXTERIOR; }
    return LEAN ? compact_locate_lean((const dv2*)(d.compact + 16 * ci), x, y, poly)
                : compact_locate((const dv2*)(d.compact + 16 * ci), x, y, poly);
  }
  if (GM_REF_BAD((uint64_t)ref >= (uint64_t)d.n_blob16)) { pip_fault(d, PIP_FAULT_BLOB); poly = -1; return LOC_EXTERIOR; }
  const double* b = d.blob + 2 * (uint64_t)ref;
  const int2 h = *(const int2*)b;
  poly = h.x;
  return blob_locate(d, b, h, x, y);
}
// ------------------------------------------------------------------ kernel LDS budgets
// The staged join (gm_pip_join.hip): one 1024-thread block per CU, per wave a fine queue and an item
// queue; what the queues leave of the 160 KiB holds the coarse EMPTY bitmap, whose block size the
// index build (make_shortcut) picks to fit.
#ifndef GM_JQ_TPB
#define GM_JQ_TPB 1024
#endif
constexpr int QTPB = GM_JQ_TPB;
constexpr int FBATCH = 64;              // fine words per round: one per lane, kept in registers
constexpr int FCAP = FBATCH + 128;     // fine queue (< FBATCH + one step's 128)
constexpr int ICAP = 128;              // item queue (two ends)
// per wave: the fine queue (x, y, row) and the item queue (x, y, row, reference)
constexpr int JQ_WAVE_LDS = FCAP * 20 + ICAP * 24;
constexpr int CM_WORDS_MAX = (163840 - (QTPB / 64) * JQ_WAVE_LDS - 256) / 4;   // 13,248 words at 1024 threads

// The row predicate (gm_pip_relate.hip): one 1024-thread block per CU whose item queues leave room
// for a coarse EMPTY bitmap in LDS: the join's (cm, CM_WORDS_MAX words) beside 64-bit-row queues of
// 192 items, or its own finer one (rm, RM_WORDS_MAX words) beside 32-bit-row queues of 128 items
// (x, y, row, reference, polygon: 28 B) when the rows fit 32 bits.
#ifndef GM_RELATE_TPB
#define GM_RELATE_TPB 1024
#endif
constexpr int RTPB = GM_RELATE_TPB;
constexpr int RQCAP32 = 128;
constexpr int RM_WORDS_MAX = (163840 - (RTPB / 64) * RQCAP32 * 28 - 256) / 4;   // 26,560 words at 1024 threads

}  // namespace gm

struct gm_pip_index {
  gm_ctx* ctx = nullptr;
  gm::PipDev dev{};
  std::vector<void*> allocs;
  int32_t n_polys = 0;
  int64_t n_entries = 0, n_boundary = 0, n_records = 0, n_slow = 0, n_cells = 0, blob_bytes = 0, n_compact = 0;
  int64_t max_bnd_per_cell = 0;   // most BOUNDARY (cell, polygon) entries of any cell (exported layout statistic)
  int64_t max_ent_per_cell = 0;   // most (cell, polygon) entries of any cell (exported layout statistic)
  int64_t n_lines = 0;            // line shortcut entries (make_shortcut)
  const int32_t* list_poly = nullptr;   // polygon of each list_ent slot (the row-wise predicate's list search)
  const void* arr[GM_PIP_INDEX_ARRAYS] = {};   // the device arrays in gm_pip_index_layout order
  int64_t arr_bytes[GM_PIP_INDEX_ARRAYS] = {};
};
