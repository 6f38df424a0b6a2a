// gm_pip.hip -- st_contains(polygon, point) join on gfx950 with JTS 1.20 semantics.
//
// Reference path: ST_Contains = geom1.contains(geom2) (geomesa-spark-jts/.../udf/SpatialRelationFunctions.scala:29)
// evaluated per candidate pair by GeoMesaJoinRelation.sweeplineJoin / OverlapAction
// (geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91, OverlapAction.scala:25-41) after grid
// partitioning (RelationUtils.scala:30-157).  JTS Geometry.contains(point): envelope covers, then
// relate -> PointLocator with the Mod-2 boundary rule; rings via RayCrossingCounter with the robust
// CGAlgorithmsDD orientation (filter + double-double).  Boundary points are NOT contained.
//
// Index (built once on the host from the polygon CSR and uploaded -- the analogue of broadcasting
// the polygon side of the join):
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
#include <math.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "gm_arrow.hpp"
#include "gm_scan.hpp"

// GM_JX_* macros are stage-ablation timing hooks that give wrong results; geomesa_amd/build.py
// refuses them for the shipped library and defines GM_PRODUCT_BUILD there, so this guard holds
#if defined(GM_PRODUCT_BUILD) && (defined(GM_JX_BLOBUNI) || defined(GM_JX_CAPS) || defined(GM_JX_NOATOMIC) || \
                                  defined(GM_JX_NOCOARSE) || defined(GM_JX_NOFINE) || defined(GM_JX_NOBLOB))
#error "GM_JX_* timing hooks are not allowed in the product build"
#endif

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
  double gx0, gy0, gx1, gy1, inv_cw, inv_ch;
  int32_t gx, gy, gxc;
  int32_t op;                    // join predicate: JOIN_CONTAINS (interior) or JOIN_INTERSECTS (not exterior)
  // reference checks: every blob / line / list reference a kernel follows is bounded by these sizes
  // (make_shortcut); a reference beyond them sets a PIP_FAULT_* bit in *fault (the call's scratch
  // word, null = not checked by this caller) and is treated as EXTERIOR, never dereferenced
  uint32_t* fault;
  int64_t n_line, n_compact_lines, n_blob16, n_list;
  // coarse EMPTY bitmap (make_shortcut; staged in LDS by the direct join): bit (by * cm_w + bx) set when
  // every coarse cell of block (bx, by) = coarse cells [bx << cm_shift, (bx + 1) << cm_shift) x (same
  // in y) is EMPTY; cm_words = 0: no bitmap
  const uint32_t* cm;
  int32_t cm_shift, cm_w;
  int64_t cm_words;
  // the same bitmap at the row predicate's smaller LDS budget (RELATE_CM_WORDS)
  const uint32_t* cm2;
  int32_t cm2_shift, cm2_w;
  int64_t cm2_words;
  // per polygon p, a rectangle of fine cells (x0, y0, x1, y1 inclusive; x0 > x1 = none) whose words
  // are all INTERIOR(p) (make_shortcut, k_core_*): the row predicate answers a row of polygon p inside
  // it from LDS, without the coarse and fine gathers.  n_core = 0: no table
  const ushort4* core;
  int32_t n_core;
};

enum : uint32_t { PIP_FAULT_LINE = 1, PIP_FAULT_COMPACT = 2, PIP_FAULT_BLOB = 4, PIP_FAULT_LIST = 8, PIP_FAULT_QUEUE = 16 };

__device__ __forceinline__ void pip_fault(const PipDev& d, uint32_t code) {
  if (d.fault) atomicOr(d.fault, code);
}


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

__device__ __forceinline__ int cell_of(double v, double v0, double inv, int g) {
  const double c = floor(__dmul_rn(__dsub_rn(v, v0), inv));
  if (!(c >= 0.0)) return 0;
  if (c >= (double)g) return g - 1;
  return (int)c;
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
__device__ __noinline__ int locate_ring_slab(const RingDev* __restrict__ rings, const int32_t* __restrict__ slab_off,
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
__device__ int blob_locate(const PipDev& d, const double* b, int2 h, double px, double py) {
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
#ifdef GM_JX_BLOBUNI   // timing experiment only: pieces 1-7 of the line from one wave-uniform address
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    const uint64_t a = (uint64_t)(c + 8 * LINE + i);
    const uint64_t u = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
                       (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    q[i] = *(const dv2*)u;
  }
#endif
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
// shortcut (near the line: the entry's own blob), a compact blob or a generic blob
__device__ __forceinline__ int item_locate(const PipDev& d, uint32_t ref, double x, double y, int& poly) {
  int loc = -1;
  if ((ref & BLOB_COMPACT) && d.line_ent && (ref & SC_LINE)) {
    const uint64_t li = ref & (SC_LINE - 1);
    if (li >= (uint64_t)d.n_line) { pip_fault(d, PIP_FAULT_LINE); poly = -1; return LOC_EXTERIOR; }
    const uint4 e0 = d.line_ent[2 * li], e1 = d.line_ent[2 * li + 1];
    poly = (int)e0.y;
    loc = line_locate(e0, e1, x, y, d);
    ref = e0.x & 0x3fffffffu;
  }
  if (loc >= 0) return loc;
  if (ref & BLOB_COMPACT) {
    const uint64_t ci = ref & (BLOB_COMPACT - 1);
    if (ci >= (uint64_t)d.n_compact_lines) { pip_fault(d, PIP_FAULT_COMPACT); poly = -1; return LOC_EXTERIOR; }
    return compact_locate((const dv2*)(d.compact + 16 * ci), x, y, poly);
  }
  if ((uint64_t)ref >= (uint64_t)d.n_blob16) { pip_fault(d, PIP_FAULT_BLOB); poly = -1; return LOC_EXTERIOR; }
  const double* b = d.blob + 2 * (uint64_t)ref;
  const int2 h = *(const int2*)b;
  poly = h.x;
  return blob_locate(d, b, h, x, y);
}

constexpr int JTPB = 256;             // 4 waves
#ifndef GM_JILP
#define GM_JILP 2
#endif
constexpr int JILP = GM_JILP;         // points per lane per tile (their lookups overlap)
constexpr int WCAP = 512;             // LDS pair staging per wave (4 KiB)
constexpr int QCAP = 128;             // LDS blob work queue per wave (3 KiB)
constexpr int WCAP_S = 256;           // split mode: pair staging per wave (2 KiB)
constexpr int QCAP_S = 256;           // split mode: (row, blob) work items per wave (2 KiB)
constexpr int JTILE = JTPB * JILP;

__device__ __forceinline__ int lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// one global atomic reserves the wave's staged pairs; lanes copy them out
__device__ __forceinline__ void flush_pairs(const uint32_t* wpt, const int32_t* wpl, int wn, int lane, int64_t id_base,
                                            int64_t* __restrict__ pt_ids, int32_t* __restrict__ poly_ids,
                                            int64_t cap, unsigned long long* __restrict__ counter) {
  wave_lds_sync();
  unsigned long long base = 0;
#ifdef GM_JX_NOATOMIC   // timing experiment only: no output counter (pairs land in a per-wave window)
  base = ((uint64_t)(blockIdx.x * 4 + (threadIdx.x >> 6)) * 4096) % (uint64_t)(cap > 4096 ? cap - 4096 : 1);
#else
  if (lane == 0) base = atomicAdd(counter, (unsigned long long)wn);
#endif
  base = __shfl(base, 0, 64);
  for (int j = lane; j < wn; j += 64) {
    const int64_t slot = (int64_t)base + j;
    if (slot < cap) { pt_ids[slot] = id_base + (int64_t)wpt[j]; poly_ids[slot] = wpl[j]; }
  }
  wave_lds_sync();
}

// Row-band partitioned point record (24 B): the join's input after k_band_scatter.
struct PtRec {
  double x, y;
  uint32_t idx;   // row within the chunk
  uint32_t pad;
};

// Split-pass outputs.  Every wave of the split pass owns a private segment of the work list and of
// the pair list, sized for the points it can see (its block's tiles x 64 lanes x JILP, times the
// most boundary / total entries any cell has), and appends with a wave-uniform cursor: no atomics.
// A shared head word was the bottleneck of the first split version -- one returning atomic per
// flush saturates near 88 per us chip-wide (MI355X_MICROARCH.md, dequeue row): 3.2M flushes cost
// 13 ms of the pass.  k_pip_blobs walks the segments and appends its hits to the same segment's
// pairs (an atomic on that segment's count, contended by one block only); k_pip_compact packs the
// segments into the caller's arrays.
struct SplitArgs {
  uint2* items;        // [nseg][ipw] (row, blob ref)
  uint32_t* item_cnt;  // [nseg]
  int64_t ipw;
  uint2* pairs;        // [nseg][ppw] (row, polygon)
  uint32_t* pair_cnt;  // [nseg]
  int64_t ppw;
  int64_t* pair_off;   // [nseg + 1] scanned pair counts (k_pip_compact)
  int32_t nseg;
};

// append cnt staged entries at the wave's cursor (wave-uniform), clipped to the segment capacity
__device__ __forceinline__ void append_seg(const uint2* src, int cnt, int lane, uint2* __restrict__ seg, int64_t& cur,
                                           int64_t segcap) {
  wave_lds_sync();
  for (int j = lane; j < cnt; j += 64)
    if (cur + j < segcap) seg[cur + j] = src[j];
  cur += cnt;
  wave_lds_sync();
}

// Persistent grid-stride over tiles of JTILE points; every wave works independently.
// A point's candidate work is a list of items: its cell word (INTERIOR -> match, BOUNDARY -> one
// blob), or, for a LIST cell, one item per (cell, polygon) entry.  Items are walked one per lane per
// step (wave-uniform loop): INTERIOR items emit their pair at once, blob items are compacted into a
// per-wave LDS queue (ballot + mbcnt), and whenever 64 are queued the wave evaluates them with all
// lanes busy (JTS RayCrossingCounter over the blob's segments).  This keeps the long boundary walk
// off the lanes whose points sit in uniform cells.  Pairs are staged per wave in LDS and flushed
// with one global atomic per few hundred pairs.
#ifndef GM_JOIN_WAVES
#define GM_JOIN_WAVES 1
#endif
//
// SPLIT (the direct pass): blob items are not evaluated here but appended, as (row, blob) pairs of
// 8 B, to a global work list that k_pip_blobs evaluates next.  Without the blob code the kernel fits
// 64 VGPRs and 16 KiB of LDS per block, i.e. 8 waves per SIMD instead of 4, which is what the
// lookup chain (point -> coarse word -> fine word -> list) needs to hide its latency.
// SRC: 0 = x / y columns, 1 / 2 = an Arrow point column of Float8 / Float4 tuples (ap)
template <bool WRITE, bool REC, bool SPLIT, int SRC = 0>
__global__ __launch_bounds__(JTPB, GM_JOIN_WAVES) void k_pip_join(const double* __restrict__ px, const double* __restrict__ py,
                                                   const PtRec* __restrict__ rec, const uint32_t* __restrict__ n_rec,
                                                   int64_t n, int64_t id_base, PipDev d, int64_t* __restrict__ pt_ids,
                                                   int32_t* __restrict__ poly_ids, int64_t cap,
                                                   unsigned long long* __restrict__ counter, SplitArgs sp,
                                                   ArrowPts ap) {
  constexpr int NW = JTPB / 64;
  constexpr int WC = SPLIT ? WCAP_S : WCAP;
  __shared__ uint32_t s_pt[WRITE && !SPLIT ? NW * WC : 1];
  __shared__ int32_t s_poly[WRITE && !SPLIT ? NW * WC : 1];
  __shared__ uint2 s_pp[WRITE && SPLIT ? NW * WC : 1];     // split: (row, polygon) staging
  __shared__ double s_qx[SPLIT ? 1 : NW * QCAP], s_qy[SPLIT ? 1 : NW * QCAP];
  __shared__ uint32_t s_qid[SPLIT ? 1 : NW * QCAP], s_qb[SPLIT ? 1 : NW * QCAP];
  __shared__ uint2 s_qi[SPLIT ? NW * QCAP_S : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* wpt = s_pt + (WRITE ? wv * WC : 0);
  int32_t* wpl = s_poly + (WRITE ? wv * WC : 0);
  double* qx = s_qx + (SPLIT ? 0 : wv * QCAP);
  double* qy = s_qy + (SPLIT ? 0 : wv * QCAP);
  uint32_t* qid = s_qid + (SPLIT ? 0 : wv * QCAP);
  uint32_t* qb = s_qb + (SPLIT ? 0 : wv * QCAP);
  uint2* qi = s_qi + (SPLIT ? wv * QCAP_S : 0);
  uint2* wpp = s_pp + (WRITE && SPLIT ? wv * WC : 0);
  const int64_t seg = (int64_t)blockIdx.x * NW + wv;   // split: this wave's private segments
  int64_t icur = 0, pcur = 0;
  int wn = 0, qn = 0, qg = 0;   // wave-uniform fills of the pair staging and the blob queue (compact / generic)
  int my_count = 0;
  if (REC) n = *n_rec;
  const int64_t ntiles = (n + JTILE - 1) / JTILE;
  // REC: band-sorted input -> XCD-aware mapping (workgroups are dispatched round-robin over the 8
  // XCDs): each XCD sweeps its own contiguous eighth of the records.
  int64_t tile = blockIdx.x, t_end = ntiles, t_step = gridDim.x;
  if (REC) {
    const int nx = 8, xcd = blockIdx.x % nx;
    tile = ntiles * xcd / nx + blockIdx.x / nx;
    t_end = ntiles * (xcd + 1) / nx;
    t_step = gridDim.x / nx;
  }
  for (;;) {
    const bool have = tile < t_end;   // block-uniform
    double x[JILP], y[JILP];
    uint32_t id[JILP], cw[JILP];
    int lo[JILP], ni[JILP];
    uint4 lq[JILP];
#pragma unroll
    for (int u = 0; u < JILP; ++u) {
      const int64_t i = tile * JTILE + u * JTPB + threadIdx.x;
      x[u] = y[u] = NAN;
      id[u] = (uint32_t)i;
      if (have && i < n) {
        if (REC) {
          const PtRec* r = rec + i;
          x[u] = __builtin_nontemporal_load(&r->x);
          y[u] = __builtin_nontemporal_load(&r->y);
          id[u] = __builtin_nontemporal_load(&r->idx);
        } else if (SRC != 0) {   // null slots keep NaN: no cell, no pair
          if (arrow_valid(ap.valid, ap.voff, i)) arrow_tuple<SRC == 2>(ap.c, i, ap.flip, x[u], y[u]);
        } else {
          x[u] = __builtin_nontemporal_load(&px[i]);
          y[u] = __builtin_nontemporal_load(&py[i]);
        }
      }
    }
    int cxs[JILP], cys[JILP];
#pragma unroll
    for (int u = 0; u < JILP; ++u) {
      cw[u] = CELL_EMPTY << 30;
      cxs[u] = cys[u] = 0;
      if (x[u] >= d.gx0 && x[u] <= d.gx1 && y[u] >= d.gy0 && y[u] <= d.gy1) {
        cxs[u] = cell_of(x[u], d.gx0, d.inv_cw, d.gx);
        cys[u] = cell_of(y[u], d.gy0, d.inv_ch, d.gy);
#ifdef GM_JX_NOCOARSE   // timing experiment only: no coarse lookup (every point EMPTY)
        cw[u] = CELL_EMPTY << 30;
#else
        cw[u] = coarse_mask(d.coarse_sc[(int64_t)(cys[u] >> CF_LOG) * d.gxc + (cxs[u] >> CF_LOG)], cxs[u], cys[u], d.coarse_fmt);
#endif
      }
    }
#pragma unroll
    for (int u = 0; u < JILP; ++u)
      if ((cw[u] >> 30) == CELL_LIST) {
#ifdef GM_JX_NOFINE   // timing experiment only: stop at the coarse level
        cw[u] = CELL_EMPTY << 30;
#else
        cw[u] = d.cell_sc[(int64_t)cys[u] * d.gx + cxs[u]];
#endif
      }
#pragma unroll
    for (int u = 0; u < JILP; ++u) {
      const uint32_t kind = cw[u] >> 30;
      lo[u] = 0;
      ni[u] = kind == CELL_EMPTY ? 0 : 1;
      lq[u] = make_uint4(cw[u], 0u, 0u, 0u);
      if (kind == CELL_LIST) {
        lo[u] = 4 * (int)((cw[u] & 0x3fffffffu) >> 4);
        ni[u] = (int)(cw[u] & 15u);
        if ((int64_t)lo[u] + 4 > d.n_list) { pip_fault(d, PIP_FAULT_LIST); ni[u] = 0; cw[u] = CELL_EMPTY << 30; }
        else lq[u] = *(const uint4*)(d.list_ent + lo[u]);   // the first four slots, all points at once
      }
    }
#pragma unroll
    for (int u = 0; u < JILP; ++u) {
      if (ni[u] == LIST_LONG && (cw[u] >> 30) == CELL_LIST) {   // long list: [count, entries...]
        ni[u] = (int)lq[u].x;
        lo[u] += 1;
        lq[u] = make_uint4(lq[u].y, lq[u].z, lq[u].w, 0u);
        if (ni[u] < 0 || (int64_t)lo[u] + ni[u] > d.n_list) { pip_fault(d, PIP_FAULT_LIST); ni[u] = 0; }
      }
    }
    // item walk; after the last tile the same loop drains the queue and ends
    int pre[JILP + 1];
    pre[0] = 0;
#pragma unroll
    for (int u = 0; u < JILP; ++u) pre[u + 1] = pre[u] + ni[u];
    const int ntot = pre[JILP];
    for (int k = 0;; ++k) {
      const bool act = k < ntot;
      const bool any = __ballot(act) != 0;
      if (!any && (have ? qn + qg < (SPLIT ? QCAP_S - 64 : 64) : qn + qg == 0)) break;   // split: qg = 0
      if (any) {
        // item k belongs to the last point u with pre[u] <= k (static selects, no register indexing)
        double ex = x[0], ey = y[0];
        uint32_t eid = id[0], w = cw[0];
        uint4 q = lq[0];
        int j = k, base = lo[0];
#pragma unroll
        for (int u = 1; u < JILP; ++u)
          if (k >= pre[u]) { ex = x[u]; ey = y[u]; eid = id[u]; w = cw[u]; q = lq[u]; j = k - pre[u]; base = lo[u]; }
        // slot j of the point's list: registers for the first slots, a load beyond them (long lists)
        uint32_t e = j == 0 ? q.x : j == 1 ? q.y : j == 2 ? q.z : q.w;
        if (act && (w >> 30) == CELL_LIST && j >= 3 && !(j == 3 && (w & 15u) != LIST_LONG))
          e = d.list_ent[base + j];
        const bool hit = act && (e >> 30) == CELL_INTERIOR;
        const bool blob = act && (e >> 30) != CELL_INTERIOR;
        if (!WRITE) my_count += hit;
        if (WRITE) {
          const uint64_t m = __ballot(hit);
          if (hit) {
            const int o = wn + lanes_below(m);
            if (SPLIT) wpp[o] = make_uint2(eid, e & 0x3fffffffu);
            else { wpt[o] = eid; wpl[o] = (int32_t)(e & 0x3fffffffu); }
          }
          wn += __popcll(m);
        }
        if (SPLIT) {
          const uint64_t mq = __ballot(blob);
          if (qn + 64 > QCAP_S) { if (lane == 0 && mq) pip_fault(d, PIP_FAULT_QUEUE); }   // cannot happen: qn < QCAP_S - 64 here
          else {
            if (blob) qi[qn + lanes_below(mq)] = make_uint2(eid, e & 0x3fffffffu);
            qn += __popcll(mq);
          }
        } else {
          // line-entry items stack up from slot 0, blob items (compact and generic, rare once the
          // shortcuts apply) down from slot QCAP - 1, so an evaluation round runs one kind of code
          const bool cmp = (e & (BLOB_COMPACT | SC_LINE)) == (BLOB_COMPACT | SC_LINE) && d.line_ent;
          const uint64_t mc = __ballot(blob && cmp), mg = __ballot(blob && !cmp);
          // invariant: qn + qg < 64 before a step (the evaluation below restores it), so this step's
          // <= 64 items fit the QCAP = 128 slots from both ends without meeting
          if (qn + qg + 64 > QCAP) { if (lane == 0 && (mc | mg)) pip_fault(d, PIP_FAULT_QUEUE); }
          else {
            if (blob) {
              const int o = cmp ? qn + lanes_below(mc) : QCAP - 1 - qg - lanes_below(mg);
              qx[o] = ex; qy[o] = ey; qid[o] = eid; qb[o] = e & 0x3fffffffu;
            }
            qn += __popcll(mc);
            qg += __popcll(mg);
          }
        }
      }
      if (SPLIT) {
        if (qn >= QCAP_S - 64 || (!have && !any && qn > 0)) {   // hand the wave's items to the work list
          append_seg(qi, qn, lane, sp.items + seg * sp.ipw, icur, sp.ipw);
          qn = 0;
        }
      } else if (qn + qg >= 64 || (!have && !any && qn + qg > 0)) {
        // evaluate the newest min(count, 64) items of the fuller kind: the queue then holds < 64
        // items again, whatever the mix (qn + qg < 128 here, so the fuller kind holds at least half)
        wave_lds_sync();
        const bool cmp = qn >= qg;
        const int kq = min(cmp ? qn : qg, 64);
        const int slot = cmp ? qn - kq + lane : QCAP - qg + lane;
        bool hit = false;
        int poly = 0;
        uint32_t eid = 0;
        if (lane < kq) {
          const uint32_t ref = qb[slot];
          const double ex = qx[slot], ey = qy[slot];
          eid = qid[slot];
#ifdef GM_JX_NOBLOB   // timing experiment only: no blob evaluation
          if (true) {
            poly = 0; hit = false;
          } else
#endif
          {   // one kind per round (cmp: line entries, else compact / generic blobs); item_locate takes any ref
            hit = join_hit(d.op, item_locate(d, ref, ex, ey, poly));
          }
        }
        wave_lds_sync();
        if (cmp) qn -= kq;
        else qg -= kq;
        if (!WRITE) my_count += hit;
        if (WRITE) {
          const uint64_t m = __ballot(hit);
          if (hit) { const int o = wn + lanes_below(m); wpt[o] = eid; wpl[o] = poly; }
          wn += __popcll(m);
        }
      }
      if (WRITE && wn > WC - 128) {
        if (SPLIT) append_seg(wpp, wn, lane, sp.pairs + seg * sp.ppw, pcur, sp.ppw);
        else flush_pairs(wpt, wpl, wn, lane, id_base, pt_ids, poly_ids, cap, counter);
        wn = 0;
      }
    }
    if (!have) break;
    tile += t_step;
  }
  if (WRITE && wn > 0) {
    if (SPLIT) append_seg(wpp, wn, lane, sp.pairs + seg * sp.ppw, pcur, sp.ppw);
    else flush_pairs(wpt, wpl, wn, lane, id_base, pt_ids, poly_ids, cap, counter);
  }
  if (SPLIT && lane == 0) {
    sp.item_cnt[seg] = (uint32_t)min(icur, sp.ipw);
    if (WRITE) sp.pair_cnt[seg] = (uint32_t)min(pcur, sp.ppw);
  }
  if (!WRITE) {
    for (int off = 32; off > 0; off >>= 1) my_count += __shfl_down(my_count, off, 64);
    if (lane == 0 && my_count) atomicAdd(counter, (unsigned long long)my_count);
  }
}

// ---------------------------------------------------------------- pair output by slabs
// One returning atomic on one output counter saturates near 88 per us chip-wide (MI355X_MICROARCH.md,
// "dequeue"): a flush of a few hundred staged pairs each was ~0.8M atomics per 1B-point join, several
// ms of serialised counter traffic.  Instead each wave reserves SLAB pairs at a time (one atomic per
// 4096 pairs) and writes its pairs straight into its slab, 64 at a time, no LDS staging.  Only each
// wave's last slab can be partly filled; the waves record (slab base, fill) and, after the join,
// k_pair_plan lists the holes below the pair count and the pairs at or above it, and k_pair_move
// moves those into these (at most waves x SLAB pairs): the caller gets [0, n_pairs) contiguous.
// Slab positions at or past the caller's capacity land in a context overflow area (waves x SLAB
// pairs), so nothing below n_pairs is lost when reservations run past cap while n_pairs fits.
constexpr int SLAB = 4096;
constexpr int PLAN_MAX = 8192;       // wave descriptors one plan handles

struct PairOut {
  int64_t* pt; int32_t* pl; int64_t cap;       // caller arrays
  int64_t* opt; int32_t* opl; int64_t ocap;    // overflow area: positions [cap, cap + ocap)
  unsigned long long* counter;                 // slab reservations (pairs), then the pair count
  longlong2* desc;                             // per wave: (last slab base or -1, its fill)
};

__device__ __forceinline__ void pair_store(const PairOut& o, int64_t pos, int64_t id, int32_t poly) {
  if (pos < o.cap) { o.pt[pos] = id; o.pl[pos] = poly; }
  else if (pos - o.cap < o.ocap) { o.opt[pos - o.cap] = id; o.opl[pos - o.cap] = poly; }
}

struct PairPlan {
  int64_t n_pairs, moves, n_src, n_dst;
  int64_t src[PLAN_MAX + 1], src_pre[PLAN_MAX + 2];   // source runs (start) and their exclusive prefix
  int64_t dst[PLAN_MAX + 1], dst_pre[PLAN_MAX + 2];   // hole runs below n_pairs
};

// exclusive scan of (x, y) over the 1024 threads of a block (s: 2 x 16 scratch words); totals in tot
__device__ __forceinline__ longlong2 plan_exscan(longlong2 v, int64_t* s, longlong2& tot) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int64_t x = v.x, y = v.y;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t px = __shfl_up(x, o, 64), py = __shfl_up(y, o, 64);
    if (lane >= o) { x += px; y += py; }
  }
  if (lane == 63) { s[wv] = x; s[16 + wv] = y; }
  __syncthreads();
  int64_t bx = 0, by = 0, tx = 0, ty = 0;
  for (int w = 0; w < 16; ++w) {
    if (w < wv) { bx += s[w]; by += s[16 + w]; }
    tx += s[w]; ty += s[16 + w];
  }
  __syncthreads();
  tot = make_longlong2(tx, ty);
  return make_longlong2(bx + x - v.x, by + y - v.y);
}

// one block: sort the waves' last slabs by base, then the hole runs below the pair count and the pair
// runs at or above it, with block scans (a serial walk by one thread cost 0.77 ms per join);
// counter[0] becomes the pair count
__global__ __launch_bounds__(1024) void k_pair_plan(const longlong2* __restrict__ desc, int nd,
                                                    unsigned long long* __restrict__ counter, PairPlan* __restrict__ plan) {
  constexpr int PER = PLAN_MAX / 1024;   // sorted slots per thread (contiguous)
  __shared__ int64_t key[PLAN_MAX];
  __shared__ int32_t fil[PLAN_MAX];
  __shared__ int64_t s_scan[32];
  int P = 1;
  while (P < nd) P <<= 1;
#pragma unroll 1
  for (int i = threadIdx.x; i < PLAN_MAX; i += blockDim.x) {
    const bool ok = i < nd && desc[i].x >= 0 && desc[i].y < SLAB;   // a slab with a hole
    key[i] = ok ? desc[i].x : INT64_MAX;
    fil[i] = ok ? (int32_t)desc[i].y : SLAB;
  }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          if ((key[i] > key[l]) == up) {
            const int64_t t = key[i]; key[i] = key[l]; key[l] = t;
            const int32_t f = fil[i]; fil[i] = fil[l]; fil[l] = f;
          }
        }
      }
      __syncthreads();
    }
  const int64_t T = (int64_t)*counter;
  const int i0 = (int)threadIdx.x * PER;
  // H = every hole's size (holes sort first; the rest are INT64_MAX)
  longlong2 tot;
  int64_t hsum = 0, nv = 0;
  for (int e = 0; e < PER; ++e)
    if (key[i0 + e] != INT64_MAX) { hsum += SLAB - fil[i0 + e]; ++nv; }
  (void)plan_exscan(make_longlong2(hsum, nv), s_scan, tot);
  const int64_t np = T - tot.x, nh = tot.y;
  // dst: the part of each hole below np (a prefix of the sorted holes); src: the pairs at or above np
  // between the previous hole's end (or np) and each hole's start, then the tail up to T
  // (per slot: the dst length, the src run [a, b); recomputed in the write loop, not kept)
  auto slot = [&](int i, int64_t& dl, int64_t& a, int64_t& b) {
    dl = 0; a = b = 0;
    if (i >= nh) return;
    const int64_t hs = key[i] + fil[i], he = key[i] + SLAB;
    if (hs < np) dl = min(he, np) - hs;
    if (he > np) {
      a = i > 0 ? max(np, key[i - 1] + SLAB) : np;
      b = max(a, hs);
    }
  };
  int64_t dsum = 0, dcnt = 0, ssum = 0, scnt = 0;
#pragma unroll 1
  for (int e = 0; e < PER; ++e) {
    int64_t dl, a, b;
    slot(i0 + e, dl, a, b);
    if (dl > 0) { dsum += dl; ++dcnt; }
    if (b > a) { ssum += b - a; ++scnt; }
  }
  longlong2 dt, st;
  const longlong2 dx = plan_exscan(make_longlong2(dsum, dcnt), s_scan, dt);
  const longlong2 sx = plan_exscan(make_longlong2(ssum, scnt), s_scan, st);
  int64_t dpre = dx.x, dix = dx.y, spre = sx.x, six = sx.y;
#pragma unroll 1
  for (int e = 0; e < PER; ++e) {
    const int i = i0 + e;
    int64_t dl, a, b;
    slot(i, dl, a, b);
    if (dl > 0) { plan->dst[dix] = key[i] + fil[i]; plan->dst_pre[dix] = dpre; dpre += dl; ++dix; }
    if (b > a) { plan->src[six] = a; plan->src_pre[six] = spre; spre += b - a; ++six; }
  }
  if (threadIdx.x == 0) {
    const int64_t cur = nh > 0 ? max(np, key[nh - 1] + SLAB) : np;
    int64_t ns = st.y, sacc = st.x;
    if (T > cur) { plan->src[ns] = cur; plan->src_pre[ns] = sacc; sacc += T - cur; ++ns; }
    plan->dst_pre[dt.y] = dt.x;
    plan->src_pre[ns] = sacc;
    plan->n_dst = dt.y; plan->n_src = ns;
    plan->moves = min(dt.x, sacc);   // equal by construction
    plan->n_pairs = np;
    *counter = (unsigned long long)np;
  }
}

__device__ __forceinline__ int64_t run_of(const int64_t* pre, int64_t n, int64_t k) {   // last r with pre[r] <= k
  int64_t a = 0, b = n - 1;
  while (a < b) {
    const int64_t m = (a + b + 1) >> 1;
    if (pre[m] <= k) a = m;
    else b = m - 1;
  }
  return a;
}

__global__ __launch_bounds__(256) void k_pair_move(PairOut o, const PairPlan* __restrict__ plan) {
  const int64_t L = plan->moves, np = plan->n_pairs;
  if (np > o.cap) return;   // GM_E_CAPACITY: nothing to deliver
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < L; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t rs = run_of(plan->src_pre, plan->n_src, k), rd = run_of(plan->dst_pre, plan->n_dst, k);
    const int64_t sp = plan->src[rs] + (k - plan->src_pre[rs]), dp = plan->dst[rd] + (k - plan->dst_pre[rd]);
    int64_t id;
    int32_t pl;
    if (sp < o.cap) { id = o.pt[sp]; pl = o.pl[sp]; }
    else { id = o.opt[sp - o.cap]; pl = o.opl[sp - o.cap]; }
    o.pt[dp] = id;
    o.pl[dp] = pl;
  }
}

// ---------------------------------------------------------------- the direct pass, stage queues
// The direct join as three stages joined by per-wave LDS queues, so that every gather beyond L2 is
// issued by a full wave (64 independent addresses) and many are in flight at once:
//   1. stream: a step is 128 consecutive points of the wave's stream, 2 per lane (16-B pair loads
//      of x and y; the next step's loads are issued while this one is processed).  Their coarse
//      words (L2-resident) decide INTERIOR / EMPTY coarse cells (after the sub-block masks); the
//      other points go to the fine queue F.
//   2. fine: whenever F holds 128 points, 2 per lane take their fine words (cell_sc) in one go and
//      resolve them one after the other: INTERIOR / EMPTY decide; a LINE word or a blob word becomes
//      an item; a LIST word walks its entries (INTERIOR: a pair; a blob: an item), one per lane per
//      loop trip.
//   3. items: line-entry items stack up from slot 0 of the item queue, blob items down from slot
//      ICAP - 1; whenever 64 are queued, one kind runs on all lanes: a line entry decides from its
//      quantized lines or hands its blob over as a blob item, a blob is walked (PointLocator).
// One loop runs the stages by priority (items, list walks, pending fine words, fine rounds, the
// stream), so each stage's code exists once and the queues stay bounded: the item queue holds < 64
// before any push of <= 64 (and a line round hands over at most the items it took), F < 128 before
// a stream step pushes <= 128.  Both are checked (PIP_FAULT_QUEUE).  Pairs are staged per wave and
// flushed with one atomic per flush.
// One 1024-thread block per CU (16 waves, 9 KiB of queues each) leaves 16 KiB of LDS for the coarse
// EMPTY bitmap (one bit per 2 x 2 coarse cells on the bench's index; 768 threads left 52 KiB for one
// bit per coarse cell, but 16 waves hide more: 11.45 -> 10.88 ms): a point whose coarse block is
// EMPTY costs no gather at all.  The join is bound by the
// vector-memory path (TD busy 97%, the L1 stalled on its outstanding misses 83% of the kernel, r3
// PMC), and the coarse lookups were 70% of its L1 misses; 55% of the bench's points sit in EMPTY
// coarse cells.
#ifndef GM_JQ_TPB
#define GM_JQ_TPB 1024
#endif
constexpr int QTPB = GM_JQ_TPB;
#ifndef GM_JQ_FBATCH
#define GM_JQ_FBATCH 64
#endif
constexpr int FBATCH = GM_JQ_FBATCH;   // fine words per round (64: 1 per lane, 128: 2 per lane)
constexpr int FCAP = FBATCH + 128;     // fine queue (< FBATCH + one step's 128)
constexpr int ICAP = 128;           // item queue (two ends)
// per wave: the fine queue (x, y, row; plus each point's fine word when a round resolves two halves)
// and the item queue (x, y, row, reference)
constexpr int JQ_WAVE_LDS = FCAP * (FBATCH > 64 ? 24 : 20) + ICAP * 24;
constexpr int CM_WORDS_MAX = (163840 - (QTPB / 64) * JQ_WAVE_LDS - 256) / 4;   // the rest of the 160 KiB: 4,032 words at 1024 threads

template <bool WRITE, int SRC, bool VEC>
__global__ __launch_bounds__(QTPB) void k_pip_join_q(const double* __restrict__ px, const double* __restrict__ py,
                                                     int64_t n, int64_t id_base, PipDev d, PairOut po,
                                                     int64_t desc_base, ArrowPts ap) {
  constexpr int NW = QTPB / 64;
  __shared__ double s_fx[NW][FCAP], s_fy[NW][FCAP];
  __shared__ uint32_t s_fid[NW][FCAP], s_fw[NW][FBATCH > 64 ? FCAP : 1];   // one half per round: its words stay in registers
  __shared__ double s_ix[NW][ICAP], s_iy[NW][ICAP];
  __shared__ uint32_t s_iid[NW][ICAP], s_iref[NW][ICAP];
  __shared__ uint32_t s_cm[CM_WORDS_MAX];
  const int64_t cm_words = d.cm_words <= CM_WORDS_MAX ? d.cm_words : 0;
  for (int64_t i = threadIdx.x; i < cm_words; i += QTPB) s_cm[i] = d.cm[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* fx = s_fx[wv]; double* fy = s_fy[wv]; uint32_t* fid = s_fid[wv];
  double* qx = s_ix[wv]; double* qy = s_iy[wv]; uint32_t* qid = s_iid[wv]; uint32_t* qref = s_iref[wv];
  int fn = 0, qn = 0, qg = 0;   // wave-uniform fills: fine queue, line items, blob items
  int64_t sbase = -1;           // wave-uniform: this wave's current output slab and its fill
  int sfill = SLAB;
  int my_count = 0;
  const bool lines_on = d.line_ent != nullptr;

  // a wave's pairs go straight into its slab (see "pair output by slabs"); a full slab takes the
  // next one with one atomic
  auto pair_push = [&](bool hit, uint32_t id, int poly) __attribute__((always_inline)) {
    if (!WRITE) { my_count += hit; return; }
    const uint64_t m = __ballot(hit);
    if (!m) return;
    const int c = __popcll(m), off = lanes_below(m), room = SLAB - sfill;
    if (hit && off < room) pair_store(po, sbase + sfill + off, id_base + id, poly);
    if (c > room) {
      unsigned long long b = 0;
      if (lane == 0) b = atomicAdd(po.counter, (unsigned long long)SLAB);
      sbase = (int64_t)__shfl(b, 0, 64);
      if (hit && off >= room) pair_store(po, sbase + (off - room), id_base + id, poly);
      sfill = c - room;
    } else {
      sfill += c;
    }
  };
  auto item_push = [&](bool valid, bool is_line, double x, double y, uint32_t id, uint32_t ref) __attribute__((always_inline)) {
    const uint64_t ml = __ballot(valid && is_line), mb = __ballot(valid && !is_line);
    if (!(ml | mb)) return;
    if (qn + qg + 64 > ICAP) { if (lane == 0) pip_fault(d, PIP_FAULT_QUEUE); return; }   // cannot happen: < 64 here
    if (valid) {
      const int o = is_line ? qn + lanes_below(ml) : ICAP - 1 - qg - lanes_below(mb);
      qx[o] = x; qy[o] = y; qid[o] = id; qref[o] = ref;
    }
    qn += __popcll(ml);
    qg += __popcll(mb);
  };

  // stream: step k of this wave covers pairs [k * 64, k * 64 + 64) of its share, 2 points per lane
  const int64_t npair = (n + 1) >> 1;
  const int64_t nstep = (npair + 63) >> 6;
  const int64_t wstride = (int64_t)gridDim.x * NW;
  int64_t step = (int64_t)blockIdx.x * NW + wv;
  auto load_pair = [&](int64_t k, double& x0, double& x1, double& y0, double& y1) __attribute__((always_inline)) {
    const int64_t i = 2 * (k * 64 + lane);
    x0 = x1 = y0 = y1 = NAN;
    if (k >= nstep) return;
    if (SRC == 0) {
      if (VEC && i + 1 < n) {
        const dv2 a = __builtin_nontemporal_load((const dv2*)(px + i));
        const dv2 b = __builtin_nontemporal_load((const dv2*)(py + i));
        x0 = a.x; x1 = a.y; y0 = b.x; y1 = b.y;
      } else {
        if (i < n) { x0 = px[i]; y0 = py[i]; }
        if (i + 1 < n) { x1 = px[i + 1]; y1 = py[i + 1]; }
      }
    } else {   // Arrow tuples; null slots keep NaN (no cell, no pair)
      if (i < n && arrow_valid(ap.valid, ap.voff, i)) arrow_tuple<SRC == 2>(ap.c, i, ap.flip, x0, y0);
      if (i + 1 < n && arrow_valid(ap.valid, ap.voff, i + 1)) arrow_tuple<SRC == 2>(ap.c, i + 1, ap.flip, x1, y1);
    }
  };
  double X0, X1, Y0, Y1, NX0, NX1, NY0, NY1;
  load_pair(step, X0, X1, Y0, Y1);
  load_pair(step + wstride, NX0, NX1, NY0, NY1);

  // pending fine words: a fine round leaves its window [pb, pb + pc) of the fine queue in place and
  // stores each point's word beside it (s_fw); the window is resolved in two halves of 64 and only
  // then released.  The list walk of a half reads its point back from the window.
  int pb = 0, pc = 0, hn = 0, hd = 0;   // wave-uniform: window base and size, next half, halves
  bool list_on = false;              // wave-uniform: some lane walks a list
  int l_slot = 0, l_lo = 0, l_n = 0, l_j = 0;
  uint32_t* fw = s_fw[wv];
  uint32_t pend_w = CELL_EMPTY << 30;   // FBATCH == 64: the pending window's word of this lane

  for (;;) {
    // every other stage idle: the item stage drains what is left (a line round may hand blobs over)
    const bool idle = !list_on && hn == hd && fn == 0 && step >= nstep;
    if (qn + qg >= 64 || (idle && qn + qg > 0)) {   // ---- items: one round of the fuller kind
      wave_lds_sync();
      const bool lines = qn >= qg;
      const int kq = min(lines ? qn : qg, 64);
      const int slot = lines ? qn - kq + lane : ICAP - qg + lane;
      const bool act = lane < kq;
      double x = 0.0, y = 0.0;
      uint32_t id = 0, ref = 0;
      if (act) { x = qx[slot]; y = qy[slot]; id = qid[slot]; ref = qref[slot]; }
      wave_lds_sync();
      if (lines) qn -= kq;
      else qg -= kq;
      int poly = 0;
      if (lines) {
        int loc = -1;
        uint32_t blob = 0;
        if (act) {
          const uint64_t li = ref & (SC_LINE - 1);
          if (li >= (uint64_t)d.n_line) { pip_fault(d, PIP_FAULT_LINE); loc = LOC_EXTERIOR; }
          else {
            const uint4 e0 = d.line_ent[2 * li], e1 = d.line_ent[2 * li + 1];
            poly = (int)e0.y;
            loc = line_locate(e0, e1, x, y, d);
            blob = e0.x & 0x3fffffffu;
          }
        }
        pair_push(act && loc >= 0 && join_hit(d.op, loc), id, poly);
        // near a line: the entry's own blob, as a blob item (fits: at most kq were taken)
        const bool fb = act && loc < 0;
        const uint64_t mb = __ballot(fb);
        if (fb) {
          const int o = ICAP - 1 - qg - lanes_below(mb);
          qx[o] = x; qy[o] = y; qid[o] = id; qref[o] = blob;
        }
        qg += __popcll(mb);
      } else {
        const int loc = act ? item_locate(d, ref, x, y, poly) : LOC_EXTERIOR;
        pair_push(act && join_hit(d.op, loc), id, poly);
      }
      continue;
    }
    if (list_on) {   // ---- one entry of each walking lane's list
      const bool act = l_j < l_n;
      const uint32_t e = act ? d.list_ent[l_lo + l_j] : (CELL_EMPTY << 30);
      double x = 0.0, y = 0.0;
      uint32_t id = 0;
      if (act) { x = fx[l_slot]; y = fy[l_slot]; id = fid[l_slot]; }
      pair_push(act && (e >> 30) == CELL_INTERIOR, id, (int)(e & 0x3fffffffu));
      item_push(act && (e >> 30) == CELL_BOUNDARY, false, x, y, id, e & 0x3fffffffu);
      ++l_j;
      list_on = __ballot(l_j < l_n) != 0;
      continue;
    }
    if (hn < hd) {   // ---- resolve one half of the pending window
      const int slot = pb + hn * 64 + lane;
      const bool act = slot < pb + pc;
      ++hn;
      uint32_t w = CELL_EMPTY << 30, id = 0;
      double x = 0.0, y = 0.0;
      if (act) { w = FBATCH > 64 ? fw[slot] : pend_w; x = fx[slot]; y = fy[slot]; id = fid[slot]; }
      const uint32_t kind = w >> 30, ref = w & 0x3fffffffu;
      pair_push(kind == CELL_INTERIOR, id, (int)ref);
      const bool item = kind == CELL_BOUNDARY;
      item_push(item, item && lines_on && (ref & (BLOB_COMPACT | SC_LINE)) == (BLOB_COMPACT | SC_LINE), x, y, id, ref);
      l_j = 0;
      l_n = 0;
      if (kind == CELL_LIST) {
        l_slot = slot;
        l_lo = 4 * (int)(ref >> 4);
        l_n = (int)(w & 15u);
        if ((int64_t)l_lo + 4 > d.n_list) { pip_fault(d, PIP_FAULT_LIST); l_n = 0; }
        else if (l_n == LIST_LONG) { l_n = (int)d.list_ent[l_lo]; l_lo += 1; }
        if (l_n < 0 || (int64_t)l_lo + l_n > d.n_list) { pip_fault(d, PIP_FAULT_LIST); l_n = 0; }
      }
      list_on = __ballot(l_j < l_n) != 0;
      if (hn == hd) fn = pb;  // the window is released once its last half is resolved (list walks
                              // of that half run next, before anything can push to the queue)
      continue;
    }
    const bool streaming = step < nstep;
    if (fn >= FBATCH || (!streaming && fn > 0)) {   // ---- fine round: the newest min(fn, 128) points
      wave_lds_sync();
      const int cnt = min(fn, FBATCH);
      const int a = fn - cnt + lane, b = a + 64;
      const bool act_a = lane < cnt, act_b = FBATCH > 64 && lane + 64 < cnt;
      uint32_t wa = CELL_EMPTY << 30, wb = CELL_EMPTY << 30;
      if (act_a) wa = d.cell_sc[(int64_t)cell_of(fy[a], d.gy0, d.inv_ch, d.gy) * d.gx + cell_of(fx[a], d.gx0, d.inv_cw, d.gx)];
      if (act_b) wb = d.cell_sc[(int64_t)cell_of(fy[b], d.gy0, d.inv_ch, d.gy) * d.gx + cell_of(fx[b], d.gx0, d.inv_cw, d.gx)];
      if (FBATCH > 64) {
        if (act_a) fw[a] = wa;
        if (act_b) fw[b] = wb;
      } else {
        pend_w = wa;
      }
      wave_lds_sync();
      pb = fn - cnt;
      pc = cnt;
      hn = 0;
      hd = cnt > 64 ? 2 : 1;
      continue;
    }
    if (streaming) {   // ---- stream step: 2 points per lane, their coarse words together
      uint32_t c0 = CELL_EMPTY << 30, c1 = CELL_EMPTY << 30;
      int cx0 = 0, cy0 = 0, cx1 = 0, cy1 = 0;
      bool g0 = X0 >= d.gx0 && X0 <= d.gx1 && Y0 >= d.gy0 && Y0 <= d.gy1;   // NaN fails
      bool g1 = X1 >= d.gx0 && X1 <= d.gx1 && Y1 >= d.gy0 && Y1 <= d.gy1;
      if (g0) { cx0 = cell_of(X0, d.gx0, d.inv_cw, d.gx); cy0 = cell_of(Y0, d.gy0, d.inv_ch, d.gy); }
      if (g1) { cx1 = cell_of(X1, d.gx0, d.inv_cw, d.gx); cy1 = cell_of(Y1, d.gy0, d.inv_ch, d.gy); }
      if (cm_words) {   // EMPTY coarse blocks from the LDS bitmap: no gather
        const int b0 = ((cy0 >> CF_LOG) >> d.cm_shift) * d.cm_w + ((cx0 >> CF_LOG) >> d.cm_shift);
        const int b1 = ((cy1 >> CF_LOG) >> d.cm_shift) * d.cm_w + ((cx1 >> CF_LOG) >> d.cm_shift);
        const bool e0 = (s_cm[b0 >> 5] >> (b0 & 31)) & 1u, e1 = (s_cm[b1 >> 5] >> (b1 & 31)) & 1u;
        g0 = g0 && !e0;
        g1 = g1 && !e1;
      }
      if (g0) c0 = d.coarse_sc[(int64_t)(cy0 >> CF_LOG) * d.gxc + (cx0 >> CF_LOG)];
      if (g1) c1 = d.coarse_sc[(int64_t)(cy1 >> CF_LOG) * d.gxc + (cx1 >> CF_LOG)];
      c0 = coarse_mask(c0, cx0, cy0, d.coarse_fmt);
      c1 = coarse_mask(c1, cx1, cy1, d.coarse_fmt);
      const uint32_t id0 = (uint32_t)(2 * (step * 64 + lane)), id1 = id0 + 1;
      pair_push((c0 >> 30) == CELL_INTERIOR, id0, (int)(c0 & 0x3fffffffu));
      pair_push((c1 >> 30) == CELL_INTERIOR, id1, (int)(c1 & 0x3fffffffu));
      const bool f0 = (c0 >> 30) == CELL_LIST, f1 = (c1 >> 30) == CELL_LIST;
      const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
      if (fn + 128 > FCAP) { if (lane == 0 && (m0 | m1)) pip_fault(d, PIP_FAULT_QUEUE); }   // cannot happen: fn < 128
      else {
        if (f0) { const int o = fn + lanes_below(m0); fx[o] = X0; fy[o] = Y0; fid[o] = id0; }
        fn += __popcll(m0);
        if (f1) { const int o = fn + lanes_below(m1); fx[o] = X1; fy[o] = Y1; fid[o] = id1; }
        fn += __popcll(m1);
      }
      step += wstride;
      X0 = NX0; X1 = NX1; Y0 = NY0; Y1 = NY1;
      load_pair(step + wstride, NX0, NX1, NY0, NY1);
      continue;
    }
    break;   // every stage idle and the item queue empty (the item stage drains it once nothing else runs)
  }
  if (WRITE) {
    if (lane == 0) po.desc[desc_base + (int64_t)blockIdx.x * NW + wv] = make_longlong2(sbase, sfill);
  } else {
    for (int off = 32; off > 0; off >>= 1) my_count += __shfl_down(my_count, off, 64);
    if (lane == 0 && my_count) atomicAdd(po.counter, (unsigned long long)my_count);
  }
}

// Evaluation of the split pass's work list: one (row, blob) item per lane, every lane busy with
// the same kind of work (JTS RayCrossingCounter over the blob's segments, compact or generic).
// The row's coordinates are re-read from the point columns; items come in roughly ascending row
// order (per wave and tile), so those reads stay within few lines per wave.
template <bool WRITE>
__global__ __launch_bounds__(JTPB) void k_pip_blobs(const double* __restrict__ px, const double* __restrict__ py,
                                                    PipDev d, unsigned long long* __restrict__ counter, SplitArgs sp) {
  constexpr int NW = JTPB / 64;
  __shared__ uint2 s_pp[WRITE ? NW * WCAP : 1];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint2* wpp = s_pp + (WRITE ? wv * WCAP : 0);
  int my_count = 0;
  for (int64_t seg = blockIdx.x; seg < sp.nseg; seg += gridDim.x) {   // block-uniform
    const uint2* items = sp.items + seg * sp.ipw;
    const int64_t n = sp.item_cnt[seg];
    int wn = 0;
    for (int64_t b0 = wv * 64; b0 < n; b0 += JTPB) {   // wave-uniform
      const int64_t i = b0 + lane;
      bool hit = false;
      int poly = 0;
      uint32_t row = 0;
      if (i < n) {
        const uint2 it = items[i];
        row = it.x;
        const uint32_t ref = it.y;
        hit = join_hit(d.op, item_locate(d, ref, px[row], py[row], poly));
      }
      if (!WRITE) my_count += hit;
      if (WRITE) {
        const uint64_t m = __ballot(hit);
        if (hit) wpp[wn + lanes_below(m)] = make_uint2(row, (uint32_t)poly);
        wn += __popcll(m);
        if (wn > WCAP - 64 || b0 + JTPB >= n) {   // the segment's last step flushes too
          if (wn > 0) {
            wave_lds_sync();
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&sp.pair_cnt[seg], (uint32_t)wn);
            base = __shfl(base, 0, 64);
            uint2* dst = sp.pairs + seg * sp.ppw;
            for (int j = lane; j < wn; j += 64)
              if ((int64_t)base + j < sp.ppw) dst[base + j] = wpp[j];
            wave_lds_sync();
          }
          wn = 0;
        }
      }
    }
  }
  if (!WRITE) {
    for (int off = 32; off > 0; off >>= 1) my_count += __shfl_down(my_count, off, 64);
    if (lane == 0 && my_count) atomicAdd(counter, (unsigned long long)my_count);
  }
}

// exclusive scan of the segments' pair counts (one block); total -> pair_off[nseg]
__global__ __launch_bounds__(1024) void k_pip_scan_segs(SplitArgs sp) {
  __shared__ int64_t part[1024];
  const int t = threadIdx.x;
  const int64_t len = sp.nseg, per = (len + 1023) / 1024, lo = t * per, hi = min(len, lo + per);
  int64_t s = 0;
  for (int64_t k = lo; k < hi; ++k) s += min((int64_t)sp.pair_cnt[k], sp.ppw);
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;
  for (int64_t k = lo; k < hi; ++k) { sp.pair_off[k] = run; run += min((int64_t)sp.pair_cnt[k], sp.ppw); }
  if (t == 1023) sp.pair_off[len] = part[1023];
}

// packs the segments into the caller's arrays after the pairs of earlier chunks (counter[0]);
// pairs beyond cap are counted, not written
__global__ __launch_bounds__(JTPB) void k_pip_compact(SplitArgs sp, const unsigned long long* __restrict__ counter,
                                                      int64_t id_base, int64_t* __restrict__ pt_ids,
                                                      int32_t* __restrict__ poly_ids, int64_t cap) {
  const int64_t base = (int64_t)*counter;
  for (int64_t seg = blockIdx.x; seg < sp.nseg; seg += gridDim.x) {
    const int64_t o = base + sp.pair_off[seg], k = sp.pair_off[seg + 1] - sp.pair_off[seg];
    const uint2* src = sp.pairs + seg * sp.ppw;
    for (int64_t j = threadIdx.x; j < k; j += JTPB) {
      const uint2 pr = src[j];
      if (o + j < cap) { pt_ids[o + j] = id_base + (int64_t)pr.x; poly_ids[o + j] = (int32_t)pr.y; }
    }
  }
}

__global__ void k_pip_chunk_done(SplitArgs sp, unsigned long long* __restrict__ counter) {
  if (threadIdx.x == 0) *counter += (unsigned long long)sp.pair_off[sp.nseg];
}

// ------------------------------------------------------------------ row-band partition
// Large joins first group the points by horizontal band of grid rows (a one-pass counting sort,
// the device analogue of RelationUtils.grid's shuffle of both sides into grid cells,
// geomesa-spark-sql/.../RelationUtils.scala:30-157).  A band's cell words and blobs then stay
// L2-resident while the join sweeps its points.  Points whose y is outside the grid (or NaN) are
// dropped here: no polygon can contain them.
constexpr int NBAND = 256;          // max bands (band id fits LDS histograms of one wave-multiple)
constexpr int PTPB = 256;           // partition block
constexpr int PTILE = 2048;         // scatter tile: 8 points per thread, sorted by band in LDS

// Coarse triage (the partition pass resolves what the coarse table already decides): a point
// outside the grid or in an EMPTY coarse cell is dropped (band nb), a point in an INTERIOR coarse
// cell is a final pair with the cell's polygon (band nb, *w = the coarse word), and only points in
// mixed (LIST) coarse cells become records of their row band for the join pass.
__device__ __forceinline__ int triage_band(double x, double y, uint32_t w, const PipDev& d, int rows_per_band, int nb) {
  if ((w >> 30) != CELL_LIST) return nb;
  return cell_of(y, d.gy0, d.inv_ch, d.gy) / rows_per_band;
}

// the coarse word of a point (EMPTY outside the grid / NaN)
__device__ __forceinline__ uint32_t coarse_of(double x, double y, const PipDev& d) {
  if (!(x >= d.gx0 && x <= d.gx1 && y >= d.gy0 && y <= d.gy1)) return CELL_EMPTY << 30;
  const int cx = cell_of(x, d.gx0, d.inv_cw, d.gx), cy = cell_of(y, d.gy0, d.inv_ch, d.gy);
  return coarse_mask(d.coarse_sc[(int64_t)(cy >> CF_LOG) * d.gxc + (cx >> CF_LOG)], cx, cy, d.coarse_fmt);
}

// per-block band histogram of the triaged points, band-major: hist[band * gridDim.x + block], and
// the block's count of coarse-INTERIOR pairs: pcount[block]
__global__ __launch_bounds__(PTPB) void k_band_hist(const double* __restrict__ px, const double* __restrict__ py,
                                                    int64_t n, int64_t per_block, PipDev d, int rows_per_band, int nb,
                                                    uint32_t* __restrict__ hist, uint32_t* __restrict__ pcount) {
  constexpr int U = PTILE / PTPB;
  __shared__ uint32_t h[NBAND + 1];
  __shared__ uint32_t s_pairs;
  for (int b = threadIdx.x; b <= nb; b += PTPB) h[b] = 0;
  if (threadIdx.x == 0) s_pairs = 0;
  __syncthreads();
  uint32_t pairs = 0;
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(n, b0 + per_block);
  for (int64_t t0 = b0; t0 < b1; t0 += PTILE) {
    double x[U], y[U];
    uint32_t w[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int64_t j = t0 + k * PTPB + threadIdx.x;
      x[k] = y[k] = NAN;
      if (j < b1) { x[k] = __builtin_nontemporal_load(&px[j]); y[k] = __builtin_nontemporal_load(&py[j]); }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) w[k] = coarse_of(x[k], y[k], d);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int b = triage_band(x[k], y[k], w[k], d, rows_per_band, nb);
      if (b < nb) atomicAdd(&h[b], 1u);
      pairs += (w[k] >> 30) == CELL_INTERIOR;
    }
  }
  for (int off = 32; off > 0; off >>= 1) pairs += __shfl_down(pairs, off, 64);
  if ((threadIdx.x & 63) == 0 && pairs) atomicAdd(&s_pairs, pairs);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += PTPB) hist[(int64_t)b * gridDim.x + blockIdx.x] = h[b];
  if (threadIdx.x == 0) pcount[blockIdx.x] = s_pairs;
}

// in-place exclusive scan of hist[0, len) by one 1024-thread block; hist[len] = total kept points.
// The blocks' coarse-INTERIOR pair counts pcount[0, nblk) become their output slots after the pairs
// already counted (*counter), and *counter moves past them (the join pass appends after).
__global__ __launch_bounds__(1024) void k_band_scan(uint32_t* __restrict__ hist, int64_t len, uint32_t* __restrict__ pcount,
                                                    int nblk, int64_t* __restrict__ poff,
                                                    unsigned long long* __restrict__ counter) {
  __shared__ uint32_t part[1024];
  const int t = threadIdx.x;
  const int64_t per = (len + 1023) / 1024, a = t * per, b = min(len, a + per);
  uint32_t s = 0;
  for (int64_t k = a; k < b; ++k) s += hist[k];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const uint32_t v = t >= off ? part[t - off] : 0u;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - s;
  for (int64_t k = a; k < b; ++k) { const uint32_t c = hist[k]; hist[k] = run; run += c; }
  if (t == 1023) hist[len] = part[1023];
  __syncthreads();
  if (t < 64) {   // nblk is small (one resident wave of partition blocks): one wave scans it
    const unsigned long long base = *counter;
    unsigned long long run2 = 0;
    for (int c0 = 0; c0 < nblk; c0 += 64) {
      const int j = c0 + t;
      const unsigned long long v = j < nblk ? pcount[j] : 0ull;
      unsigned long long inc = v;
      for (int o = 1; o < 64; o <<= 1) { const unsigned long long u = __shfl_up(inc, o, 64); if (t >= o) inc += u; }
      if (j < nblk) poff[j] = (int64_t)(base + run2 + inc - v);
      run2 += __shfl(inc, 63, 64);
    }
    if (t == 0) *counter = base + run2;
  }
}

// Scatter: tile of PTILE points -> coarse triage -> coarse-INTERIOR pairs written at the block's
// pair slots, LIST points counting-sorted by band in LDS -> each band's run written as consecutive
// 24-B records at the block's running cursor for that band.
template <bool WRITE>
__global__ __launch_bounds__(PTPB) void k_band_scatter(const double* __restrict__ px, const double* __restrict__ py,
                                                       int64_t n, int64_t per_block, PipDev d, int rows_per_band,
                                                       int nb, const uint32_t* __restrict__ off,
                                                       PtRec* __restrict__ rec, const int64_t* __restrict__ poff,
                                                       int64_t id_base, int64_t* __restrict__ pt_ids,
                                                       int32_t* __restrict__ poly_ids, int64_t cap) {
  constexpr int PER_T = PTILE / PTPB;
  __shared__ uint32_t cnt[NBAND + 1], loff[NBAND + 2], gcur[NBAND];
  __shared__ double sx[PTILE], sy[PTILE];
  __shared__ uint32_t sid[PTILE];
  __shared__ uint16_t sband[PTILE];
  __shared__ uint32_t s_np;
  const int t = threadIdx.x;
  for (int b = t; b <= nb; b += PTPB) cnt[b] = 0;
  for (int b = t; b < nb; b += PTPB) gcur[b] = off[(int64_t)b * gridDim.x + blockIdx.x];
  if (t == 0) s_np = 0;
  int64_t pbase = WRITE ? poff[blockIdx.x] : 0;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * per_block, b1 = min(n, b0 + per_block);
  for (int64_t t0 = b0; t0 < b1; t0 += PTILE) {
    double x[PER_T], y[PER_T];
    int band[PER_T];
    uint32_t r[PER_T], w[PER_T];
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
      const int64_t j = t0 + k * PTPB + t;
      x[k] = y[k] = NAN;
      if (j < b1) { x[k] = __builtin_nontemporal_load(&px[j]); y[k] = __builtin_nontemporal_load(&py[j]); }
    }
#pragma unroll
    for (int k = 0; k < PER_T; ++k) w[k] = coarse_of(x[k], y[k], d);
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
      const int64_t j = t0 + k * PTPB + t;
      band[k] = -1;
      if (j < b1) {
        band[k] = triage_band(x[k], y[k], w[k], d, rows_per_band, nb);
        r[k] = atomicAdd(&cnt[band[k]], 1u);
        if (WRITE && (w[k] >> 30) == CELL_INTERIOR) {
          const int64_t slot = pbase + atomicAdd(&s_np, 1u);
          if (slot < cap) { pt_ids[slot] = id_base + j; poly_ids[slot] = (int32_t)(w[k] & 0x3fffffffu); }
        }
      }
    }
    __syncthreads();
    if (WRITE) pbase += s_np;
    if (t < 64) {   // exclusive scan of cnt[0..nb] by one wave
      constexpr int PER_L = (NBAND + 1 + 63) / 64;
      uint32_t v[PER_L], s = 0;
#pragma unroll
      for (int k = 0; k < PER_L; ++k) { const int b = t * PER_L + k; v[k] = b <= nb ? cnt[b] : 0u; s += v[k]; }
      uint32_t inc = s;
      for (int o = 1; o < 64; o <<= 1) { const uint32_t w = __shfl_up(inc, o, 64); if (t >= o) inc += w; }
      uint32_t run = inc - s;
#pragma unroll
      for (int k = 0; k < PER_L; ++k) { const int b = t * PER_L + k; if (b <= nb) loff[b] = run; run += v[k]; }
      if (t == 63) loff[nb + 1] = inc;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER_T; ++k) {
      if (band[k] < 0 || band[k] == nb) continue;   // dropped or resolved by the triage
      const uint32_t pos = loff[band[k]] + r[k];
      sx[pos] = x[k]; sy[pos] = y[k];
      sid[pos] = (uint32_t)(t0 + k * PTPB + t);
      sband[pos] = (uint16_t)band[k];
    }
    __syncthreads();
    const int kept = (int)loff[nb];   // drop bin sorts last
    for (int q = t; q < kept; q += PTPB) {
      const int b = sband[q];
      PtRec* o = rec + gcur[b] + (q - loff[b]);
      o->x = sx[q]; o->y = sy[q];
      *(uint2*)&o->idx = make_uint2(sid[q], 0u);
    }
    __syncthreads();
    for (int b = t; b <= nb; b += PTPB) {
      if (b < nb) gcur[b] += cnt[b];
      cnt[b] = 0;
    }
    if (t == 0) s_np = 0;
    __syncthreads();
  }
}

// ------------------------------------------------------------------ host-side JTS (index build)
namespace host {

static int sgn(double x) { return x > 0 ? 1 : (x < 0 ? -1 : 0); }

// CGAlgorithmsDD.orientationIndex (filter + DD), host copy for the index build
static int orientation(double p1x, double p1y, double p2x, double p2y, double qx, double qy) {
  volatile double detleft = (p1x - qx) * (p2y - qy);
  volatile double detright = (p1y - qy) * (p2x - qx);
  double det = detleft - detright, detsum;
  if (detleft > 0.0) {
    if (detright <= 0.0) return sgn(det);
    detsum = detleft + detright;
  } else if (detleft < 0.0) {
    if (detright >= 0.0) return sgn(det);
    detsum = -detleft - detright;
  } else {
    return sgn(det);
  }
  double errbound = 1e-15 * detsum;
  if ((det >= errbound) || (-det >= errbound)) return sgn(det);
  auto add_d = [](double hi, double lo, double y, double& rhi, double& rlo) {
    double S = hi + y, e = S - hi, s = S - e;
    s = (y - e) + (hi - s);
    double f = s + lo, H = S + f, h = f + (S - H);
    rhi = H + h;
    rlo = h + (H - rhi);
  };
  auto mul = [](double hi, double lo, double yhi, double ylo, double& rhi, double& rlo) {
    const double SPLIT = 134217729.0;
    double C = SPLIT * hi, hx = C - hi, c = SPLIT * yhi;
    hx = C - hx;
    double tx = hi - hx, hy = c - yhi;
    C = hi * yhi;
    hy = c - hy;
    double ty = yhi - hy;
    c = ((((hx * hy - C) + hx * ty) + tx * hy) + tx * ty) + (hi * ylo + lo * yhi);
    double zhi = C + c;
    hx = C - zhi;
    rhi = zhi;
    rlo = c + hx;
  };
  double a1, a2, b1, b2, c1, c2, d1, d2, ah, al, bh, bl;
  add_d(p2x, 0.0, -p1x, a1, a2);
  add_d(p2y, 0.0, -p1y, b1, b2);
  add_d(qx, 0.0, -p2x, c1, c2);
  add_d(qy, 0.0, -p2y, d1, d2);
  mul(a1, a2, d1, d2, ah, al);
  mul(b1, b2, c1, c2, bh, bl);
  double yhi = -bh, ylo = -bl;
  double S = ah + yhi, T = al + ylo, e = S - ah, f = T - al, s = S - e, t = T - f;
  s = (yhi - e) + (ah - s);
  t = (ylo - f) + (al - t);
  e = s + T;
  double H = S + e, h = e + (S - H);
  e = t + h;
  double zhi = H + e, zlo = e + (H - zhi);
  if (zhi > 0.0) return 1;
  if (zhi < 0.0) return -1;
  if (zlo > 0.0) return 1;
  if (zlo < 0.0) return -1;
  return 0;
}

static int locate_ring(const double* vx, const double* vy, int n, double px, double py) {
  if (n < 1) return LOC_EXTERIOR;
  double mnx = vx[0], mxx = vx[0], mny = vy[0], mxy = vy[0];
  for (int i = 1; i < n; ++i) {
    mnx = std::min(mnx, vx[i]); mxx = std::max(mxx, vx[i]);
    mny = std::min(mny, vy[i]); mxy = std::max(mxy, vy[i]);
  }
  if (!(px >= mnx && px <= mxx && py >= mny && py <= mxy)) return LOC_EXTERIOR;
  int crossings = 0;
  for (int i = 1; i < n; ++i) {
    double p1x = vx[i], p1y = vy[i], p2x = vx[i - 1], p2y = vy[i - 1];
    if (p1x < px && p2x < px) continue;
    if (px == p2x && py == p2y) return LOC_BOUNDARY;
    if (p1y == py && p2y == py) {
      double mn = std::min(p1x, p2x), mx = std::max(p1x, p2x);
      if (px >= mn && px <= mx) return LOC_BOUNDARY;
      continue;
    }
    if (((p1y > py) && (p2y <= py)) || ((p2y > py) && (p1y <= py))) {
      int o = orientation(p1x, p1y, p2x, p2y, px, py);
      if (o == 0) return LOC_BOUNDARY;
      if (p2y < p1y) o = -o;
      if (o == 1) crossings++;
    }
  }
  return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

static int locate_poly(const gm_polyset* ps, int poly, double px, double py) {
  bool is_in = false;
  int nb = 0;
  for (int p = ps->poly_part_off[poly]; p < ps->poly_part_off[poly + 1]; ++p) {
    const int r0 = ps->part_ring_off[p], r1 = ps->part_ring_off[p + 1];
    if (r1 <= r0) continue;
    const int v0 = ps->ring_vert_off[r0], v1 = ps->ring_vert_off[r0 + 1];
    int loc = locate_ring(ps->vx + v0, ps->vy + v0, v1 - v0, px, py);
    if (loc == LOC_INTERIOR) {
      for (int r = r0 + 1; r < r1; ++r) {
        const int h0 = ps->ring_vert_off[r], h1 = ps->ring_vert_off[r + 1];
        const int hl = locate_ring(ps->vx + h0, ps->vy + h0, h1 - h0, px, py);
        if (hl == LOC_INTERIOR) { loc = LOC_EXTERIOR; break; }
        if (hl == LOC_BOUNDARY) { loc = LOC_BOUNDARY; break; }
      }
    }
    if (loc == LOC_INTERIOR) is_in = true;
    if (loc == LOC_BOUNDARY) nb++;
  }
  if (nb & 1) return LOC_BOUNDARY;
  if (nb > 0 || is_in) return LOC_INTERIOR;
  return LOC_EXTERIOR;
}

static inline int cell_of(double v, double v0, double inv, int g) {
  volatile double t = (v - v0) * inv;  // keep the exact device op order (sub, mul, floor)
  double c = floor(t);
  if (!(c >= 0.0)) return 0;
  if (c >= (double)g) return g - 1;
  return (int)c;
}

}  // namespace host
}  // namespace gm

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

template <int OP>
__device__ __forceinline__ bool entry_pred(const PipDev& d, uint32_t e, double px, double py) {
  if ((e >> 30) == CELL_INTERIOR) return true;   // every point of the cell is interior
  const uint32_t ref = e & 0x3fffffffu;
  if (!blob_ref_ok(d, ref)) { pip_fault(d, PIP_FAULT_BLOB); return false; }
  int loc;
  if (ref & BLOB_COMPACT) {
    int poly;
    loc = compact_locate((const dv2*)(d.compact + 16 * (uint64_t)(ref & (BLOB_COMPACT - 1))), px, py, poly);
  } else {
    const double* b = d.blob + 2 * (uint64_t)ref;
    loc = blob_locate(d, b, *(const int2*)b, px, py);
  }
  return OP == SP_INTERSECTS ? loc != LOC_EXTERIOR : loc == LOC_INTERIOR;
}

// Phases per lane, over the lane's 2 * FPAIRS rows:
//  1. the streaming terms (16-B loads, registers only); rows inside the index envelope keep their
//     coarse and fine cell numbers;
//  2. the coarse words of all surviving rows, then the fine words of those in LIST coarse cells --
//     independent loads issued together, so the chain costs two L2 round trips per lane, not two
//     per row;
//  3. the rows still undecided (boundary cells, multi-polygon lists) walk their blobs one per loop
//     trip, re-reading the row's coordinates (keeping the staged columns live through the walk
//     costs 32 VGPRs).
#ifndef GM_QUERY_WAVES
#define GM_QUERY_WAVES 1
#endif
template <bool VEC, bool DURING, int OP>
__global__ __launch_bounds__(FTPB, GM_QUERY_WAVES) void k_query_mask(const double* __restrict__ x, const double* __restrict__ y,
                                                     const int64_t* __restrict__ t, int64_t n, int has_bbox,
                                                     double bx0, double by0, double bx1, double by1, int64_t lo,
                                                     int64_t hi, PipDev d, uint64_t* __restrict__ mask,
                                                     int32_t* __restrict__ block_counts) {
  constexpr int R = 2 * FPAIRS;
  const int64_t npairs = n >> 1, nwords = (n + 63) >> 6;
  const int wave = threadIdx.x >> 6;
  const int64_t pbase = (int64_t)blockIdx.x * (FTPB * FPAIRS);
  dv2 xv[FPAIRS], yv[FPAIRS];
  lv2 tv[FPAIRS];
  uint32_t live = 0;   // bit 2u + j: row j of pair step u exists
#pragma unroll
  for (int u = 0; u < FPAIRS; ++u) {
    const int64_t p = pbase + (int64_t)u * FTPB + threadIdx.x;
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
  int fc[R], cc[R];   // fine / coarse cell of each row (geometry term only)
  auto cheap = [&](double px, double py, int64_t tt, int k) {
    bool ok = !has_bbox || (px >= bx0 && px <= bx1 && py >= by0 && py <= by1);
    if (DURING) ok = ok && tt > lo && tt < hi;
    if (OP != SP_NONE) {
      ok = ok && px >= d.gx0 && px <= d.gx1 && py >= d.gy0 && py <= d.gy1;
      const int cx = cell_of(px, d.gx0, d.inv_cw, d.gx), cy = cell_of(py, d.gy0, d.inv_ch, d.gy);
      fc[k] = cy * d.gx + cx;
      cc[k] = (cy >> CF_LOG) * d.gxc + (cx >> CF_LOG);
    }
    return ok;
  };
#pragma unroll
  for (int u = 0; u < FPAIRS; ++u) {
    pass |= (uint32_t)cheap(xv[u].x, yv[u].x, tv[u].x, 2 * u) << (2 * u);
    pass |= (uint32_t)cheap(xv[u].y, yv[u].y, tv[u].y, 2 * u + 1) << (2 * u + 1);
  }
  pass &= live;
  if (OP != SP_NONE && pass) {
    uint32_t cw[R];
#pragma unroll
    for (int k = 0; k < R; ++k) cw[k] = ((pass >> k) & 1u) ? d.coarse_word[cc[k]] : (CELL_EMPTY << 30);
#pragma unroll
    for (int k = 0; k < R; ++k)
      if ((cw[k] >> 30) == CELL_LIST) cw[k] = d.cell_word[fc[k]];
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
      const int64_t row = 2 * (pbase + (int64_t)(k >> 1) * FTPB + threadIdx.x) + (k & 1);
      const double px = x[row], py = y[row];
      bool hit;
      if ((w >> 30) == CELL_LIST) {
        int l0 = 4 * (int)((w & 0x3fffffffu) >> 4), ni = (int)(w & 15u);
        if ((int64_t)l0 + 4 > d.n_list) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
        else if (ni == LIST_LONG) { ni = (int)d.list_ent[l0]; l0 += 1; }
        if (ni < 0 || (int64_t)l0 + ni > d.n_list) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
        hit = false;
        for (int j = 0; j < ni && !hit; ++j) hit = entry_pred<OP>(d, d.list_ent[l0 + j], px, py);
      } else {
        hit = entry_pred<OP>(d, w, px, py);
      }
      if (!hit) pass &= ~(1u << k);
    }
  }
  int cnt = 0;
#pragma unroll
  for (int u = 0; u < FPAIRS; ++u) {
    const uint64_t be = __ballot((pass >> (2 * u)) & 1u), bo = __ballot((pass >> (2 * u + 1)) & 1u);
    cnt += __popcll(be) + __popcll(bo);
    put_pair_words(be, bo, mask, ((pbase + (int64_t)u * FTPB + wave * 64) * 2) >> 6, nwords);
  }
  block_count_waves(cnt, block_counts);
}

// ------------------------------------------------------------------ lookup census (diagnostic)
// How the join's lookup chain resolves a batch of points, stage by stage (gm_pip_join_census): the
// design numbers behind its gather costs.  Counters (JC_*) are summed per block in LDS.
enum : int {
  JC_POINTS = 0, JC_OUTSIDE, JC_COARSE_EMPTY, JC_COARSE_INTERIOR, JC_COARSE_RAW_MIXED, JC_FINE, JC_FINE_EMPTY,
  JC_FINE_INTERIOR, JC_FINE_LINE, JC_FINE_COMPACT, JC_FINE_GENERIC, JC_FINE_LIST, JC_LIST_ENTRIES,
  JC_LIST_BLOBS, JC_LINE_RESOLVED, JC_LINE_FALLBACK, JC_N
};

__global__ __launch_bounds__(256) void k_pip_census(const double* __restrict__ px, const double* __restrict__ py, int64_t n,
                                                    PipDev d, unsigned long long* __restrict__ out) {
  __shared__ unsigned long long s_c[JC_N];
  if (threadIdx.x < JC_N) s_c[threadIdx.x] = 0;
  __syncthreads();
  int c[JC_N];
#pragma unroll
  for (int k = 0; k < JC_N; ++k) c[k] = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double x = px[i], y = py[i];
    c[JC_POINTS]++;
    if (!(x >= d.gx0 && x <= d.gx1 && y >= d.gy0 && y <= d.gy1)) { c[JC_OUTSIDE]++; continue; }
    const int cx = cell_of(x, d.gx0, d.inv_cw, d.gx), cy = cell_of(y, d.gy0, d.inv_ch, d.gy);
    const uint32_t raw = d.coarse_sc[(int64_t)(cy >> CF_LOG) * d.gxc + (cx >> CF_LOG)];
    if ((raw >> 30) == CELL_LIST) c[JC_COARSE_RAW_MIXED]++;
    uint32_t w = coarse_mask(raw, cx, cy, d.coarse_fmt);
    if ((w >> 30) == CELL_EMPTY) { c[JC_COARSE_EMPTY]++; continue; }
    if ((w >> 30) == CELL_INTERIOR) { c[JC_COARSE_INTERIOR]++; continue; }
    c[JC_FINE]++;
    w = d.cell_sc[(int64_t)cy * d.gx + cx];
    const uint32_t kind = w >> 30, ref = w & 0x3fffffffu;
    if (kind == CELL_EMPTY) { c[JC_FINE_EMPTY]++; continue; }
    if (kind == CELL_INTERIOR) { c[JC_FINE_INTERIOR]++; continue; }
    if (kind == CELL_BOUNDARY) {
      if ((ref & BLOB_COMPACT) && (ref & SC_LINE) && d.line_ent && (uint64_t)(ref & (SC_LINE - 1)) < (uint64_t)d.n_line) {
        c[JC_FINE_LINE]++;
        const uint64_t li = ref & (SC_LINE - 1);
        const int l = line_locate(d.line_ent[2 * li], d.line_ent[2 * li + 1], x, y, d);
        if (l >= 0) c[JC_LINE_RESOLVED]++;
        else c[JC_LINE_FALLBACK]++;
      } else if (ref & BLOB_COMPACT) {
        c[JC_FINE_COMPACT]++;
      } else {
        c[JC_FINE_GENERIC]++;
      }
      continue;
    }
    c[JC_FINE_LIST]++;
    int l0 = 4 * (int)(ref >> 4), ni = (int)(w & 15u);
    if ((int64_t)l0 + 4 > d.n_list) ni = 0;
    else if (ni == LIST_LONG) { ni = (int)d.list_ent[l0]; l0 += 1; }
    if (ni < 0 || (int64_t)l0 + ni > d.n_list) ni = 0;
    c[JC_LIST_ENTRIES] += ni;
    for (int j = 0; j < ni; ++j) c[JC_LIST_BLOBS] += (d.list_ent[l0 + j] >> 30) != CELL_INTERIOR;
  }
#pragma unroll
  for (int k = 0; k < JC_N; ++k) {
    unsigned long long v = (unsigned long long)c[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&s_c[k], v);
  }
  __syncthreads();
  if (threadIdx.x < JC_N && s_c[threadIdx.x]) atomicAdd(&out[threadIdx.x], s_c[threadIdx.x]);
}

// ------------------------------------------------------------------ row-wise predicate (UDF path)
// st_contains / st_covers / st_intersects / ... evaluated row by row, as Spark SQL runs the UDF when
// the join rule does not apply (SpatialRelationFunctions.scala:29-37 over nullableUDF,
// SQLFunctionHelper.scala:27-33): row i pairs polygon poly[i] with point i.  Every DE-9IM predicate
// of an areal geometry and a point is a function of the point's location in the polygon
// (PointLocator.locate), so the kernel writes that location (LOC_*) and the host maps it.
// The lookup is the join's: cell word chain, then only the entry of polygon poly[i] -- INTERIOR
// decides at once, a blob is walked; no entry means the cell misses the polygon (exterior).
#ifndef GM_RELATE_TPB
#define GM_RELATE_TPB 1024
#endif
constexpr int RTPB = GM_RELATE_TPB;   // row-predicate threads per block
constexpr uint8_t LOC_NULL = 0xff;

__device__ __forceinline__ int entry_poly(const PipDev& d, uint32_t e) {
  const uint32_t ref = e & 0x3fffffffu;
  if ((e >> 30) == CELL_INTERIOR) return (int)ref;
  if (!blob_ref_ok(d, ref)) return -1;
  if (ref & BLOB_COMPACT) return (int)__double_as_longlong(d.compact[16 * (uint64_t)(ref & (BLOB_COMPACT - 1))]);
  return ((const int2*)(d.blob + 2 * (uint64_t)ref))->x;
}

__device__ __forceinline__ int entry_locate(const PipDev& d, uint32_t e, double px, double py) {
  if ((e >> 30) == CELL_INTERIOR) return LOC_INTERIOR;
  const uint32_t ref = e & 0x3fffffffu;
  if (!blob_ref_ok(d, ref)) { pip_fault(d, PIP_FAULT_BLOB); return LOC_EXTERIOR; }
  if (ref & BLOB_COMPACT) {
    int poly;
    return compact_locate((const dv2*)(d.compact + 16 * (uint64_t)(ref & (BLOB_COMPACT - 1))), px, py, poly);
  }
  const double* b = d.blob + 2 * (uint64_t)ref;
  return blob_locate(d, b, *(const int2*)b, px, py);
}

__global__ __launch_bounds__(RTPB) void k_list_poly(PipDev d, int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * RTPB + threadIdx.x;
  if (i < n) out[i] = entry_poly(d, d.list_ent[i]);   // count / padding slots read as INTERIOR: no load
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
constexpr int RELATE_CM_WORDS = 4032;   // the row predicate's bitmap budget (16 KiB)
#ifndef GM_RELATE_CORE_MAX
#define GM_RELATE_CORE_MAX 4096
#endif
constexpr int RELATE_CORE_MAX = GM_RELATE_CORE_MAX;   // polygons whose core rectangle fits LDS (8 B each)
#ifndef GM_RELATE_SPEC
#define GM_RELATE_SPEC 0
#endif
// rows that the LDS tests leave load their fine word beside the coarse word (one round trip instead
// of two for rows in mixed coarse cells, a wasted fine load for the others)
constexpr bool RELATE_SPEC = GM_RELATE_SPEC;

// VEC: a lane's RILP = 2 rows are adjacent (one 16-B load per coordinate column, one 8-B id load, one
// 2-B location store when both resolve at once); the host picks it when the columns are aligned
template <bool VEC>
__global__ __launch_bounds__(RTPB) void k_pip_relate(const int32_t* __restrict__ poly, const double* __restrict__ px,
                                                     const double* __restrict__ py, int64_t n, int32_t n_polys,
                                                     PipDev d, const int32_t* __restrict__ list_poly,
                                                     uint8_t* __restrict__ loc) {
  static_assert(!VEC || RILP == 2, "adjacent rows per lane are written for RILP = 2");
  constexpr int NW = RTPB / 64;
  __shared__ double s_x[NW][RQCAP], s_y[NW][RQCAP];
  __shared__ int64_t s_row[NW][RQCAP];
  __shared__ uint32_t s_e[NW][RQCAP];
  __shared__ int32_t s_p[NW][RQCAP];
  // the coarse EMPTY bitmap at this kernel's budget (d.cm2, 16 KiB), staged in LDS like
  // k_pip_join_q's: rows in EMPTY coarse blocks skip the coarse gather
  __shared__ uint32_t s_cm[RELATE_CM_WORDS];
  // each polygon's core rectangle (d.core): a row inside its own polygon's core is INTERIOR at once
  __shared__ ushort4 s_core[RELATE_CORE_MAX > 0 ? RELATE_CORE_MAX : 1];
  const int64_t cm_words = d.cm2_words <= RELATE_CM_WORDS ? d.cm2_words : 0;
  for (int64_t i = threadIdx.x; i < cm_words; i += RTPB) s_cm[i] = d.cm2[i];
  const int n_core = d.core && d.n_core == n_polys && d.n_core <= RELATE_CORE_MAX ? d.n_core : 0;
  for (int i = threadIdx.x; i < n_core; i += RTPB) s_core[i] = d.core[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double* qx = s_x[wave]; double* qy = s_y[wave];
  int64_t* qr = s_row[wave]; uint32_t* qe = s_e[wave]; int32_t* qp = s_p[wave];
  int qn = 0, qg = 0;   // queued line-entry items (from slot 0 up) and blob items (from RQCAP - 1 down)
  const int64_t wstep = (int64_t)gridDim.x * NW * (64 * RILP);
  for (int64_t w0 = ((int64_t)blockIdx.x * NW + wave) * (64 * RILP);; w0 += wstep) {
    const bool have = w0 < n;   // uniform per wave
    if (have) {
      int64_t row[RILP];
      int p[RILP];
      double x[RILP], y[RILP];
      uint32_t w[RILP], fw[RILP];
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
#pragma unroll
      for (int u = 0; u < RILP; ++u) {
        w[u] = CELL_EMPTY << 30;
        if (p[u] >= 0 && p[u] < n_polys && x[u] >= d.gx0 && x[u] <= d.gx1 && y[u] >= d.gy0 && y[u] <= d.gy1) {
          cx[u] = cell_of(x[u], d.gx0, d.inv_cw, d.gx);
          cy[u] = cell_of(y[u], d.gy0, d.inv_ch, d.gy);
          bool empty = false, core = false;
          if (n_core) {
            const ushort4 b = s_core[p[u]];
            core = cx[u] >= b.x && cx[u] <= b.z && cy[u] >= b.y && cy[u] <= b.w;
          }
          if (cm_words && !core) {
            const int b = ((cy[u] >> CF_LOG) >> d.cm2_shift) * d.cm2_w + ((cx[u] >> CF_LOG) >> d.cm2_shift);
            empty = (s_cm[b >> 5] >> (b & 31)) & 1u;
          }
          if (core)
            w[u] = (CELL_INTERIOR << 30) | (uint32_t)p[u];   // what the coarse word of a core cell says
          else if (!empty) {
            const uint32_t craw = d.coarse_sc[(int64_t)(cy[u] >> CF_LOG) * d.gxc + (cx[u] >> CF_LOG)];
            if (RELATE_SPEC) fw[u] = d.cell_sc[(int64_t)cy[u] * d.gx + cx[u]];   // in flight beside the coarse word
            w[u] = coarse_mask(craw, cx[u], cy[u], d.coarse_fmt);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < RILP; ++u)
        if ((w[u] >> 30) == CELL_LIST) w[u] = RELATE_SPEC ? fw[u] : d.cell_sc[(int64_t)cy[u] * d.gx + cx[u]];   // boundary shortcuts applied
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
          if ((int64_t)l0 + 4 > d.n_list) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
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
          if (ni < 0 || (int64_t)l0 + ni > d.n_list) { pip_fault(d, PIP_FAULT_LIST); ni = 0; }
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
          const int o = ln ? qn + lanes_below(ml) : RQCAP - 1 - qg - lanes_below(mb);
          qx[o] = x[u]; qy[o] = y[u]; qr[o] = row[u]; qe[o] = e; qp[o] = p[u];
        }
        qn += __popcll(ml);
        qg += __popcll(mb);
      }
      if (VEC) {
        if (dir[0] && dir[1]) *(uint16_t*)(loc + row[0]) = (uint16_t)(rv[0] | (rv[1] << 8));
        else {
          if (dir[0]) loc[row[0]] = rv[0];
          if (dir[1]) loc[row[1]] = rv[1];
        }
      }
    }
    // walk min(qn, 64) queued blobs when the queue holds a full wave, and drain it at the end
    // (< 64 queued before a step's <= 64 * RILP rows, so both ends fit RQCAP; the fuller kind goes
    // first, which leaves < 64 again)
    while (qn + qg >= 64 || (!have && qn + qg > 0)) {
      wave_lds_sync();
      const bool lines = qn >= qg;
      const int kq = min(lines ? qn : qg, 64);
      const int slot = lines ? qn - kq + lane : RQCAP - qg + lane;
      if (lane < kq) {
        const uint32_t ref = qe[slot] & 0x3fffffffu;
        const double ex = qx[slot], ey = qy[slot];
        int pl = -1;
        const int l = item_locate(d, ref, ex, ey, pl);
        loc[qr[slot]] = (uint8_t)(pl == qp[slot] ? l : LOC_EXTERIOR);
      }
      wave_lds_sync();
      if (lines) qn -= kq;
      else qg -= kq;
    }
    if (!have) break;
  }
}

template <bool VEC, bool DURING>
void launch_query(hipStream_t s, unsigned grid, int op, const double* x, const double* y, const int64_t* t, int64_t n,
                  int has_bbox, const double* bb, int64_t lo, int64_t hi, const PipDev& d, uint64_t* mask,
                  int32_t* counts) {
  switch (op) {
    case SP_INTERSECTS:
      hipLaunchKernelGGL((k_query_mask<VEC, DURING, SP_INTERSECTS>), dim3(grid), dim3(FTPB), 0, s, x, y, t, n, has_bbox,
                         bb[0], bb[1], bb[2], bb[3], lo, hi, d, mask, counts);
      break;
    case SP_CONTAINS:
      hipLaunchKernelGGL((k_query_mask<VEC, DURING, SP_CONTAINS>), dim3(grid), dim3(FTPB), 0, s, x, y, t, n, has_bbox,
                         bb[0], bb[1], bb[2], bb[3], lo, hi, d, mask, counts);
      break;
    default:
      hipLaunchKernelGGL((k_query_mask<VEC, DURING, SP_NONE>), dim3(grid), dim3(FTPB), 0, s, x, y, t, n, has_bbox,
                         bb[0], bb[1], bb[2], bb[3], lo, hi, d, mask, counts);
  }
}

}  // namespace gm

// ------------------------------------------------------------------ index build on the device
// The same classification as the host build below (gm_pip_index_create_ex), one workgroup per task
// = (polygon, grid row): the row band's ring segments are gathered in ring / vertex order (LDS, or a
// global slice for polygons with more edges than BAND_LDS), then every cell of the row is tested
// against them in parallel; the cells that no segment meets take the location of their run's first
// cell centre (PointLocator, probed once per run as on the host); boundary cells get a compact or a
// generic blob.  A count pass sizes every slot (cell of a task), a scan turns the sizes into offsets
// in slot order -- the host build's polygon / row / column order -- and the write pass fills the
// blobs, so the arrays are byte-identical to the host build's.
namespace gm {

constexpr int BT_TPB = 256;
constexpr int BAND_LDS = 1024;   // band segments kept in LDS; larger polygons use a global slice
constexpr int BUILD_MAXR = 512;  // rings per polygon handled on the device
constexpr int BUILD_MAXBK = 64;  // breakpoints collected per (cell, ring): more = slow ring

struct BandView {
  int32_t* seg;      // global vertex id of the segment end
  int32_t* ring;     // ring list index k
  double* minx;
  double* maxx;
  double* ymin;
  double* ymax;
};

struct BuildArgs {
  const int32_t* poly_part_off;
  const int32_t* part_ring_off;
  const int32_t* ring_vert_off;
  const double* vx;
  const double* vy;
  const RingDev* rings;
  const double* env;            // 4 per polygon
  const int32_t* task_poly;
  const int32_t* task_cy;
  const int64_t* task_slot;     // [ntask + 1]
  const int64_t* band_off;      // per task: global band slice offset, -1 = LDS
  BandView band_g;
  double G0, G1, inv_cw, inv_ch, epsx, epsy;
  int gx, gy;
  int write;
  int32_t* gen_words;           // count pass: generic blob words (even) per slot
  int32_t* cmp_lines;           // count pass: compact lines per slot
  const int64_t* gen_off;       // write pass: word offset per slot
  const int64_t* cmp_off;       // write pass: line offset per slot
  uint32_t* ent_word;           // write pass: entry word per slot (0xffffffff = none)
  int32_t* ent_cell;
  double* blob;
  double* compact;
  unsigned long long* stat;     // count pass: [0] slow rings, [1] ring records, [2] boundary, [3] compact
};

__device__ __forceinline__ int ring_locate_dev(const BuildArgs& a, int r, double px, double py) {
  const RingDev rd = a.rings[r];
  const int v0 = a.ring_vert_off[r], v1 = a.ring_vert_off[r + 1];
  if (v1 - v0 < 1) return LOC_EXTERIOR;
  if (!(px >= rd.minx && px <= rd.maxx && py >= rd.miny && py <= rd.maxy)) return LOC_EXTERIOR;
  int crossings = 0;
  for (int i = v0 + 1; i < v1; ++i)
    if (count_segment(a.vx[i], a.vy[i], a.vx[i - 1], a.vy[i - 1], px, py, crossings)) return LOC_BOUNDARY;
  return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

// PointLocator.locate(point, polygon): parts (shell, then holes) with the Mod-2 rule across parts
__device__ int poly_locate_dev(const BuildArgs& a, int poly, double px, double py) {
  bool is_in = false;
  int nb = 0;
  for (int q = a.poly_part_off[poly]; q < a.poly_part_off[poly + 1]; ++q) {
    const int r0 = a.part_ring_off[q], r1 = a.part_ring_off[q + 1];
    if (r1 <= r0) continue;
    int loc = ring_locate_dev(a, r0, px, py);
    if (loc == LOC_INTERIOR) {
      for (int r = r0 + 1; r < r1; ++r) {
        const int hl = ring_locate_dev(a, r, px, py);
        if (hl == LOC_INTERIOR) { loc = LOC_EXTERIOR; break; }
        if (hl == LOC_BOUNDARY) { loc = LOC_BOUNDARY; break; }
      }
    }
    if (loc == LOC_INTERIOR) is_in = true;
    if (loc == LOC_BOUNDARY) nb++;
  }
  if (nb & 1) return LOC_BOUNDARY;
  if (nb > 0 || is_in) return LOC_INTERIOR;
  return LOC_EXTERIOR;
}

// breakpoints of (cell, ring k): y of right-of-cell segment end points in (yb0, yb1], ascending,
// unique (host collect_breakpoints); returns the count, > BUILD_MAXBK - 1 when there are more
__device__ int cell_breakpoints(const BandView& b, int s0, int s1, double xb1, double yb0, double yb1, double* bk) {
  int n = 0;
  for (int s = s0; s < s1; ++s) {
    if (!(b.minx[s] > xb1)) continue;
    const double ys[2] = {b.ymin[s], b.ymax[s]};
    for (int e = 0; e < 2; ++e) {
      const double y = ys[e];
      if (!(y > yb0 && y <= yb1)) continue;
      int j = 0;   // insertion into the sorted unique list
      while (j < n && bk[j] < y) ++j;
      if (j < n && bk[j] == y) continue;
      if (n >= BUILD_MAXBK) return BUILD_MAXBK;   // too many: the ring is slow
      for (int m = n; m > j; --m) bk[m] = bk[m - 1];
      bk[j] = y;
      ++n;
    }
  }
  return n;
}

// parity of right-of-cell segments straddling y (ymin <= y < ymax) at each breakpoint interval's
// left end (host right_parity)
__device__ uint64_t cell_parity(const BandView& b, int s0, int s1, double xb1, double yb0, const double* bk, int nbk) {
  uint64_t parity = 0;
  for (int j = 0; j <= nbk; ++j) {
    const double yk = j == 0 ? yb0 : bk[j - 1];
    int c = 0;
    for (int s = s0; s < s1; ++s)
      if (b.minx[s] > xb1) c += (b.ymin[s] <= yk && yk < b.ymax[s]);
    if (c & 1) parity |= 1ull << j;
  }
  return parity;
}

__device__ __forceinline__ double i32x2_word(int32_t lo, int32_t hi) {
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

__global__ __launch_bounds__(BT_TPB) void k_build_rows(BuildArgs a) {
  __shared__ int32_t l_seg[BAND_LDS], l_ring[BAND_LDS];
  __shared__ double l_minx[BAND_LDS], l_maxx[BAND_LDS], l_ymin[BAND_LDS], l_ymax[BAND_LDS];
  __shared__ int32_t s_ring_id[BUILD_MAXR], s_bstart[BUILD_MAXR + 1];
  __shared__ uint8_t s_shell[BUILD_MAXR];
  __shared__ int32_t s_wcnt[BT_TPB / 64];
  __shared__ int s_nr, s_changed;
  __shared__ uint8_t s_bnd[BT_TPB];
  __shared__ int32_t s_probe[BT_TPB];
  __shared__ int8_t s_loc[BT_TPB];
  const int task = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int p = a.task_poly[task], cy = a.task_cy[task];
  const double* e = a.env + 4 * (int64_t)p;
  const int cx0 = cell_of(e[0], a.G0, a.inv_cw, a.gx), cx1 = cell_of(e[2], a.G0, a.inv_cw, a.gx);
  const double yb0 = __dsub_rn(__dadd_rn(a.G1, __ddiv_rn((double)cy, a.inv_ch)), a.epsy);
  const double yb1 = __dadd_rn(__dadd_rn(a.G1, __ddiv_rn((double)(cy + 1), a.inv_ch)), a.epsy);
  const int64_t slot0 = a.task_slot[task];
  BandView b;
  if (a.band_off[task] < 0) {
    b = BandView{l_seg, l_ring, l_minx, l_maxx, l_ymin, l_ymax};
  } else {
    const int64_t o = a.band_off[task];
    b = BandView{a.band_g.seg + o, a.band_g.ring + o, a.band_g.minx + o, a.band_g.maxx + o, a.band_g.ymin + o,
                 a.band_g.ymax + o};
  }
  // ring list of the polygon (RingRef order of the host build)
  if (t == 0) {
    int nr = 0;
    for (int q = a.poly_part_off[p]; q < a.poly_part_off[p + 1]; ++q)
      for (int r = a.part_ring_off[q]; r < a.part_ring_off[q + 1]; ++r) {
        if (nr < BUILD_MAXR) { s_ring_id[nr] = r; s_shell[nr] = r == a.part_ring_off[q]; }
        ++nr;
      }
    s_nr = nr;
  }
  __syncthreads();
  const int nr = s_nr;   // <= BUILD_MAXR (the host checks)
  // band: per ring, the segments whose y-range meets the row band, in vertex order
  int nb = 0;
  for (int k = 0; k < nr; ++k) {
    if (t == 0) s_bstart[k] = nb;
    const int r = s_ring_id[k];
    const int v0 = a.ring_vert_off[r], v1 = a.ring_vert_off[r + 1];
    for (int c = v0 + 1; c < v1; c += BT_TPB) {
      const int i = c + t;
      bool in = false;
      double ya = 0, yb = 0;
      if (i < v1) {
        ya = a.vy[i - 1]; yb = a.vy[i];
        const double ymn = ya < yb ? ya : yb, ymx = ya < yb ? yb : ya;
        in = !(ymx < yb0 || ymn > yb1);
      }
      const uint64_t m = __ballot(in);
      if (lane == 0) s_wcnt[wave] = __popcll(m);
      __syncthreads();
      int pre = 0, tot = 0;
      for (int w = 0; w < BT_TPB / 64; ++w) { if (w < wave) pre += s_wcnt[w]; tot += s_wcnt[w]; }
      if (in) {
        const int pos = nb + pre + __popcll(m & ((1ull << lane) - 1));
        const double xa = a.vx[i - 1], xb = a.vx[i];
        b.seg[pos] = i; b.ring[pos] = k;
        b.minx[pos] = xa < xb ? xa : xb; b.maxx[pos] = xa < xb ? xb : xa;
        b.ymin[pos] = ya < yb ? ya : yb; b.ymax[pos] = ya < yb ? yb : ya;
      }
      nb += tot;
      __syncthreads();
    }
  }
  if (t == 0) s_bstart[nr] = nb;
  __syncthreads();
  // the row's cells in segments of BT_TPB, with the run location carried between segments
  int carried = -1;   // run_loc of the host loop after the previous segment
  for (int c0 = cx0; c0 <= cx1; c0 += BT_TPB) {
    const int cx = c0 + t;
    const bool valid = cx <= cx1;
    const double xb0 = __dsub_rn(__dadd_rn(a.G0, __ddiv_rn((double)cx, a.inv_cw)), a.epsx);
    const double xb1 = __dadd_rn(__dadd_rn(a.G0, __ddiv_rn((double)(cx + 1), a.inv_cw)), a.epsx);
    bool bnd = false;
    if (valid)
      for (int s = 0; s < nb && !bnd; ++s) bnd = b.maxx[s] >= xb0 && b.minx[s] <= xb1;
    s_bnd[t] = valid ? (uint8_t)bnd : 1;
    __syncthreads();
    // probes: non-boundary cells after a boundary cell (or starting a run) locate their centre (the
    // host's run_loc < 0 case).  A probe whose centre falls outside its cell, or lands on the
    // boundary, becomes a boundary cell, which makes its successor a probe: iterate to a fixpoint
    bool probe = false, evaluated = false;
    int ploc = -1;
    for (;;) {
      if (t == 0) s_changed = 0;
      __syncthreads();
      const bool prev_bnd = t == 0 ? (carried < 0) : (s_bnd[t - 1] != 0);
      probe = valid && !s_bnd[t] && prev_bnd;
      bool fail = false;
      if (probe && !evaluated) {
        evaluated = true;
        const double cxm = __dadd_rn(a.G0, __ddiv_rn((double)cx + 0.5, a.inv_cw));
        const double cym = __dadd_rn(a.G1, __ddiv_rn((double)cy + 0.5, a.inv_ch));
        if (cell_of(cxm, a.G0, a.inv_cw, a.gx) != cx || cell_of(cym, a.G1, a.inv_ch, a.gy) != cy) fail = true;
        else {
          ploc = poly_locate_dev(a, p, cxm, cym);
          fail = ploc == LOC_BOUNDARY;
        }
      }
      __syncthreads();
      if (fail) { s_bnd[t] = 1; s_changed = 1; }
      __syncthreads();
      const int ch = s_changed;
      __syncthreads();
      if (!ch) break;
    }
    bnd = valid && s_bnd[t];
    s_loc[t] = probe ? (int8_t)ploc : (int8_t)-1;
    s_probe[t] = probe ? t : -1;
    __syncthreads();
    // last probe at or before each cell (inclusive max scan)
    for (int o = 1; o < BT_TPB; o <<= 1) {
      const int v = t >= o ? s_probe[t - o] : -1;
      __syncthreads();
      if (v > s_probe[t]) s_probe[t] = v;
      __syncthreads();
    }
    int loc = -1;
    if (valid && !bnd) loc = s_probe[t] >= 0 ? s_loc[s_probe[t]] : carried;
    // this cell's output
    const int64_t slot = slot0 + (cx - cx0);
    if (valid) {
      int gw = 0, cl = 0;
      uint32_t word = 0xffffffffu;
      const int32_t cell = cy * a.gx + cx;
      if (!bnd && loc == LOC_INTERIOR) word = (CELL_INTERIOR << 30) | (uint32_t)p;
      if (bnd) {
        double bk[BUILD_MAXBK];
        bool compact = false;
        if (nr == 1) {
          int E = 0;
          for (int s = 0; s < nb; ++s) E += (b.maxx[s] >= xb0 && b.minx[s] <= xb1);
          if (4 * E <= 30) {
            const int B = cell_breakpoints(b, 0, nb, xb1, yb0, yb1, bk);
            if (4 * E + B <= 30) {
              compact = true;
              cl = (4 * E + B <= 14 && E <= 3) ? 1 : 2;
              if (a.write) {
                double* rec = a.compact + 16 * a.cmp_off[slot];
                for (int w = 0; w < 16 * cl; ++w) rec[w] = INFINITY;
                rec[0] = i32x2_word(p, E | (cl << 8));
                rec[1] = __longlong_as_double((long long)cell_parity(b, 0, nb, xb1, yb0, bk, B));
                uint32_t used = 3u;   // word bits of the record in use
                int j = 0;
                for (int s = 0; s < nb; ++s) {
                  if (!(b.maxx[s] >= xb0 && b.minx[s] <= xb1)) continue;
                  const int i = b.seg[s], w0 = cseg_word(j);
                  rec[w0] = a.vx[i]; rec[w0 + 1] = a.vy[i]; rec[w0 + 2] = a.vx[i - 1]; rec[w0 + 3] = a.vy[i - 1];
                  used |= 15u << w0;
                  ++j;
                }
                int w = 2;
                for (int m = 0; m < B; ++m) {
                  while ((used >> w) & 1u) ++w;
                  rec[w] = bk[m];
                  used |= 1u << w;
                }
                word = (CELL_BOUNDARY << 30) | BLOB_COMPACT | (uint32_t)a.cmp_off[slot];
              } else {
                atomicAdd(&a.stat[2], 1ull);
                atomicAdd(&a.stat[3], 1ull);
              }
            }
          }
        }
        if (!compact) {
          double* out = a.write ? a.blob + a.gen_off[slot] : nullptr;
          int w = 0;
          if (out) out[w] = i32x2_word(p, nr);
          ++w;
          for (int k = 0; k < nr; ++k) {
            const int s0 = s_bstart[k], s1 = s_bstart[k + 1];
            int E = 0;
            for (int s = s0; s < s1; ++s) E += (b.maxx[s] >= xb0 && b.minx[s] <= xb1);
            const int B = cell_breakpoints(b, s0, s1, xb1, yb0, yb1, bk);
            const bool slow = E > 4096 || B > 63;
            if (out) {
              RingHdr rh{};
              rh.flags = (int16_t)((s_shell[k] ? 1 : 0) | (slow ? 2 : 0));
              rh.n_edge = slow ? 0 : (int16_t)E;
              rh.n_brk = slow ? 0 : (int16_t)B;
              double hw;
              memcpy(&hw, &rh, 8);
              out[w] = hw;
              const uint64_t par = slow ? (uint64_t)(uint32_t)s_ring_id[k] : cell_parity(b, s0, s1, xb1, yb0, bk, B);
              out[w + 1] = __longlong_as_double((long long)par);
              int q = w + 2;
              if (!slow) {
                for (int s = s0; s < s1; ++s) {
                  if (!(b.maxx[s] >= xb0 && b.minx[s] <= xb1)) continue;
                  const int i = b.seg[s];
                  out[q] = a.vx[i]; out[q + 1] = a.vy[i]; out[q + 2] = a.vx[i - 1]; out[q + 3] = a.vy[i - 1];
                  q += 4;
                }
                for (int m = 0; m < B; ++m) out[q++] = bk[m];
              }
            } else {
              if (slow) atomicAdd(&a.stat[0], 1ull);
              atomicAdd(&a.stat[1], 1ull);
            }
            w += 2 + (slow ? 0 : 4 * E + B);
          }
          gw = (w + 1) & ~1;
          if (out) {
            if (w & 1) out[w] = 0.0;
            word = (CELL_BOUNDARY << 30) | (uint32_t)(a.gen_off[slot] / 2);
          } else {
            atomicAdd(&a.stat[2], 1ull);
          }
        }
      }
      if (a.write) { a.ent_word[slot] = word; a.ent_cell[slot] = cell; }
      else { a.gen_words[slot] = gw; a.cmp_lines[slot] = cl; }
    }
    // run location after this segment's last cell
    __syncthreads();
    const int last = cx1 - c0 < BT_TPB - 1 ? cx1 - c0 : BT_TPB - 1;
    if (t == last) s_probe[0] = (valid && !bnd) ? loc : -1;   // reuse: carried run location
    __syncthreads();
    carried = s_probe[0];
    __syncthreads();
  }
}

// entries per cell (count pass over the slots)
__global__ void k_build_cell_count(const uint32_t* __restrict__ ent_word, const int32_t* __restrict__ ent_cell,
                                   int64_t nslot, int32_t* __restrict__ per_cell, int32_t* __restrict__ bnd_cell) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslot; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = ent_word[i];
    if (w == 0xffffffffu) continue;
    atomicAdd(&per_cell[ent_cell[i]], 1);
    if ((w >> 30) == CELL_BOUNDARY) atomicAdd(&bnd_cell[ent_cell[i]], 1);
  }
}

// scatter the entries into per-cell buckets (any order; sorted by polygon per cell afterwards)
__global__ void k_build_cell_scatter(const uint32_t* __restrict__ ent_word, const int32_t* __restrict__ ent_cell,
                                     int64_t nslot, const int64_t* __restrict__ cell_start, int32_t* __restrict__ fill,
                                     uint32_t* __restrict__ bucket, const int32_t* __restrict__ slot_poly) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslot; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = ent_word[i];
    if (w == 0xffffffffu) continue;
    const int c = ent_cell[i];
    const int64_t pos = cell_start[c] + atomicAdd(&fill[c], 1);
    bucket[2 * pos] = w;
    bucket[2 * pos + 1] = (uint32_t)slot_poly[i];
  }
}

// list slot count of a cell: (long-list count slot) + entries, padded to 4 (16-B aligned lists)
__device__ __forceinline__ int list_len(int k) { return k > 1 ? ((k + (k >= LIST_LONG ? 1 : 0) + 3) & ~3) : 0; }

__global__ void k_build_list_len(const int32_t* __restrict__ per_cell, int64_t ncell, int32_t* __restrict__ len) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x)
    len[c] = list_len(per_cell[c]);
}

// cell words and lists: each cell's entries sorted by polygon (the host order), single entries inline
__global__ void k_build_cells(const int32_t* __restrict__ per_cell, const int64_t* __restrict__ cell_start,
                              uint32_t* __restrict__ bucket, const int64_t* __restrict__ list_off, int64_t ncell,
                              uint32_t* __restrict__ cell_word, uint32_t* __restrict__ list_ent) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x) {
    const int k = per_cell[c];
    uint32_t* bk = bucket + 2 * cell_start[c];
    for (int i = 1; i < k; ++i) {   // insertion sort by polygon
      const uint32_t w = bk[2 * i], pl = bk[2 * i + 1];
      int j = i - 1;
      while (j >= 0 && bk[2 * j + 1] > pl) { bk[2 * (j + 1)] = bk[2 * j]; bk[2 * (j + 1) + 1] = bk[2 * j + 1]; --j; }
      bk[2 * (j + 1)] = w; bk[2 * (j + 1) + 1] = pl;
    }
    if (k == 0) { cell_word[c] = 0xffffffffu; continue; }
    if (k == 1) { cell_word[c] = bk[0]; continue; }
    const int64_t off = list_off[c];
    cell_word[c] = (CELL_LIST << 30) | (uint32_t)((off / 4) << 4) | (uint32_t)(k < LIST_LONG ? k : LIST_LONG);
    int64_t q = off;
    if (k >= LIST_LONG) list_ent[q++] = (uint32_t)k;
    for (int j = 0; j < k; ++j) list_ent[q++] = bk[2 * j];
    const int64_t end = off + list_len(k);
    while (q < end) list_ent[q++] = 0u;
  }
}

// coarse words: the fine word when every fine cell carries the same EMPTY or INTERIOR word, else LIST
__global__ void k_build_coarse(const uint32_t* __restrict__ cell_word, int gx, int gy, int gxc, int gyc,
                               uint32_t* __restrict__ coarse_word) {
  const int64_t n = (int64_t)gxc * gyc;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int yc = (int)(i / gxc), xc = (int)(i % gxc);
    uint32_t w = 0xffffffffu;
    bool first = true, mixed = false;
    for (int yy = yc << CF_LOG; yy < min(gy, (yc + 1) << CF_LOG) && !mixed; ++yy)
      for (int xx = xc << CF_LOG; xx < min(gx, (xc + 1) << CF_LOG); ++xx) {
        const uint32_t f = cell_word[(int64_t)yy * gx + xx];
        if (first) { w = f; first = false; }
        else if (f != w) { mixed = true; break; }
      }
    const uint32_t kind = w >> 30;
    coarse_word[i] = (!mixed && (kind == CELL_EMPTY || kind == CELL_INTERIOR)) ? w : (CELL_LIST << 30);
  }
}

// does segment (u1, v1)-(u2, v2) meet the box [lo, hi]^2 (cell units)?  Liang-Barsky clipping; the
// caller's box is the cell enlarged by 1% of a cell, far beyond the builder's inflation and the
// rounding of the cell-unit mapping, so "no" is certain.
__device__ __forceinline__ bool seg_meets_box(double u1, double v1, double u2, double v2, double lo, double hi) {
  double t0 = 0.0, t1 = 1.0;
  const double du = u2 - u1, dv = v2 - v1;
  const double p[4] = {-du, du, -dv, dv}, q[4] = {u1 - lo, hi - u1, v1 - lo, hi - v1};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (p[k] == 0.0) {
      if (q[k] < 0.0) return false;
    } else {
      const double r = q[k] / p[k];
      if (p[k] < 0.0) t0 = fmax(t0, r);
      else t1 = fmin(t1, r);
    }
  }
  return t0 <= t1;
}

// One cell's shortcut (see "Boundary shortcuts"): 0 = none, 1 = *word resolved to INTERIOR / EMPTY,
// 2 = a line entry in *ent.  Compact and generic blobs alike; rings left to the slab walk have no
// segment list here, so their cells keep the blob.
__device__ int analyze_cell(const PipDev& d, int64_t c, uint32_t w, uint32_t* word, uint4* ent) {
  if ((w >> 30) != CELL_BOUNDARY) return 0;
  if (!blob_ref_ok(d, w & 0x3fffffffu)) return 0;   // an out-of-range reference stays for the join to report
  if (!(isfinite(d.inv_cw) && isfinite(d.inv_ch) && d.inv_cw > 0 && d.inv_ch > 0)) return 0;
  const bool cmp = (w & BLOB_COMPACT) != 0;
  const dv2* cb = (const dv2*)(d.compact + 16 * (uint64_t)(w & (BLOB_COMPACT - 1)));
  const double* gb = d.blob + 2 * (uint64_t)(w & 0x3fffffffu);
  int poly, nseg_or_rings;
  if (cmp) {
    const int64_t meta = __double_as_longlong(cb[0].x);
    poly = (int)meta;
    nseg_or_rings = (int)((meta >> 32) & 0xff);
  } else {
    const int2 h = *(const int2*)gb;
    poly = h.x;
    nseg_or_rings = h.y;
  }
  const int cx = (int)(c % d.gx), cy = (int)(c / d.gx);
  auto cu = [&](double x) { return (x - d.gx0) * d.inv_cw - cx; };
  auto cv = [&](double y) { return (y - d.gy0) * d.inv_ch - cy; };
  // the segments crossing the enlarged cell: how many, and the first two
  int ncross = 0;
  double sg[2][4];
  auto visit = [&](double p1x, double p1y, double p2x, double p2y) -> bool {
    const double u1 = cu(p1x), v1 = cv(p1y), u2 = cu(p2x), v2 = cv(p2y);
    if (!(isfinite(u1) && isfinite(v1) && isfinite(u2) && isfinite(v2))) return false;
    if (seg_meets_box(u1, v1, u2, v2, -0.01, 1.01)) {
      if (ncross < 2) { sg[ncross][0] = u1; sg[ncross][1] = v1; sg[ncross][2] = u2; sg[ncross][3] = v2; }
      ++ncross;
    }
    return true;
  };
  if (cmp) {
    for (int j = 0; j < nseg_or_rings; ++j) {
      const dv2 s0 = cb[cseg_word(j) / 2], s1 = cb[cseg_word(j) / 2 + 1];   // p1x p1y, p2x p2y
      if (!visit(s0.x, s0.y, s1.x, s1.y)) return 0;
    }
  } else {
    const double* q = gb + 1;
    for (int r = 0; r < nseg_or_rings; ++r) {
      const RingHdr rh = *(const RingHdr*)q;
      if (rh.flags & 2) return 0;   // slab-walk ring: its segments are not in the blob
      const double* eg = q + 2;
      for (int j = 0; j < rh.n_edge; ++j)
        if (!visit(eg[4 * j], eg[4 * j + 1], eg[4 * j + 2], eg[4 * j + 3])) return 0;
      q = eg + 4 * rh.n_edge + rh.n_brk;
    }
  }
  auto locate = [&](double X, double Y) -> int {
    if (cmp) { int pp; return compact_locate(cb, X, Y, pp); }
    return blob_locate(d, gb, *(const int2*)gb, X, Y);
  };
  if (ncross == 0) {
    const double X0 = d.gx0 + (cx + 0.5) / d.inv_cw, Y0 = d.gy0 + (cy + 0.5) / d.inv_ch;
    if (cell_of(X0, d.gx0, d.inv_cw, d.gx) != cx || cell_of(Y0, d.gy0, d.inv_ch, d.gy) != cy) return 0;
    const int loc = locate(X0, Y0);   // the cell's one location
    if (loc == LOC_INTERIOR) { *word = (CELL_INTERIOR << 30) | (uint32_t)poly; return 1; }
    if (loc == LOC_EXTERIOR) { *word = CELL_EMPTY << 30; return 1; }
    return 0;
  }
  if (ncross > 2) return 0;
  uint32_t ab[2] = {0u, 0u}, cc[2] = {0u, 0u};
  for (int k = 0; k < ncross; ++k) {   // quantized line of each crossing segment
    const double u1 = sg[k][0], v1 = sg[k][1], u2 = sg[k][2], v2 = sg[k][3];
    double at = v2 - v1, bt = u1 - u2;
    const double mx = fmax(fabs(at), fabs(bt));
    if (!(mx > 0)) return 0;
    at *= 16384.0 / mx;
    bt *= 16384.0 / mx;
    const double ct = at * u1 + bt * v1;
    const double A = rint(at), B = rint(bt), C = rint(ct);
    if (!(fabs(C) < 8.0e6)) return 0;
    double dev = 0.0;
    for (int q = 0; q < 4; ++q) {
      const double uc = (q & 1) ? 1.01 : -0.01, vc = (q & 2) ? 1.01 : -0.01;
      dev = fmax(dev, fabs((A - at) * uc + (B - bt) * vc - (C - ct)));
    }
    if (!(dev <= SC_DEV)) return 0;
    ab[k] = ((uint32_t)(int32_t)A & 0xffffu) | ((uint32_t)(int32_t)B << 16);
    cc[k] = (uint32_t)(int32_t)C & 0xffffffu;
  }
  const uint4 e0 = make_uint4(w, (uint32_t)poly, ab[0], cc[0]);
  const uint4 e1 = make_uint4(ab[1], cc[1] | ((uint32_t)ncross << 24), 0u, 0u);
  uint32_t fl = 0, bad = 0;
  for (int t = 0; t < 25; ++t) {   // test points of a 5 x 5 pattern inside the cell
    const double tu = 0.04 + 0.23 * (t % 5), tv = 0.04 + 0.23 * (t / 5);
    const double X = d.gx0 + (cx + tu) / d.inv_cw, Y = d.gy0 + (cy + tv) / d.inv_ch;
    if (cell_of(X, d.gx0, d.inv_cw, d.gx) != cx || cell_of(Y, d.gy0, d.inv_ch, d.gy) != cy) continue;
    const int r = line_region(e0, e1, X, Y, d, cx, cy, 2 * SC_T);
    if (r < 0) continue;
    const int loc = locate(X, Y);
    const uint32_t has = 1u << (2 * r), in = 2u << (2 * r);
    if (loc == LOC_BOUNDARY) { bad |= has; continue; }
    const uint32_t want = loc == LOC_INTERIOR ? in : 0u;
    if ((fl & has) && (fl & in) != want) bad |= has;   // inconsistent: no shortcut for that region
    fl |= has | want;
  }
  for (int r = 0; r < 4; ++r)
    if (bad & (1u << (2 * r))) fl &= ~(3u << (2 * r));
  if (!fl) return 0;
  ent[0] = make_uint4(e0.x, e0.y, e0.z, e0.w | (fl << 24));
  ent[1] = e1;
  return 2;
}

// coarse_sc (see coarse_mask) over the resolved words cell_sc
__global__ __launch_bounds__(256) void k_build_coarse_sc(const uint32_t* __restrict__ cell_sc, int gx, int gy, int gxc,
                                                         int gyc, int32_t fmt, uint32_t* __restrict__ out) {
  const int64_t n = (int64_t)gxc * gyc;
  constexpr int CF = 1 << CF_LOG, SB = 1 << SUB_LOG;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int yc = (int)(i / gxc), xc = (int)(i % gxc);
    uint32_t w0 = 0xffffffffu, mask = 0;
    bool mixed = false;
    for (int sb = 0; sb < 16; ++sb) {
      const int x0 = xc * CF + (sb & 3) * SB, y0 = yc * CF + (sb >> 2) * SB;
      bool empty = true;
      for (int yy = y0; yy < min(gy, y0 + SB); ++yy)
        for (int xx = x0; xx < min(gx, x0 + SB); ++xx) {
          const uint32_t f = cell_sc[(int64_t)yy * gx + xx];
          if (w0 == 0xffffffffu) w0 = f;
          else if (f != w0) mixed = true;
          empty &= (f >> 30) == CELL_EMPTY;
        }
      if (empty) mask |= 1u << sb;   // (a sub-block without cells is never reached)
    }
    const uint32_t kind = w0 >> 30;
    if (fmt == COARSE_MAIN) {   // 8 sub-blocks of 4 x 2: EMPTY and INTERIOR(main) masks, main = first INTERIOR polygon
      uint32_t em = 0, im = 0, main = 0xffffffffu;
      for (int yy = yc * CF; yy < min(gy, (yc + 1) * CF) && main == 0xffffffffu; ++yy)
        for (int xx = xc * CF; xx < min(gx, (xc + 1) * CF); ++xx) {
          const uint32_t f = cell_sc[(int64_t)yy * gx + xx];
          if ((f >> 30) == CELL_INTERIOR) { main = f & 0x3fffffffu; break; }
        }
      for (int sb = 0; sb < 8; ++sb) {
        const int x0 = xc * CF + (sb & 1) * (CF / 2), y0 = yc * CF + (sb >> 1) * (CF / 4);
        bool empty = true, inner = main < (1u << 14);
        for (int yy = y0; yy < min(gy, y0 + CF / 4); ++yy)
          for (int xx = x0; xx < min(gx, x0 + CF / 2); ++xx) {
            const uint32_t f = cell_sc[(int64_t)yy * gx + xx];
            empty &= (f >> 30) == CELL_EMPTY;
            inner &= f == ((CELL_INTERIOR << 30) | main);
          }
        if (empty) em |= 1u << sb;
        else if (inner) im |= 1u << sb;
      }
      mask = em | (im << 8) | ((main < (1u << 14) ? main : 0u) << 16);
    }
    out[i] = (!mixed && (kind == CELL_EMPTY || kind == CELL_INTERIOR)) ? w0 : ((CELL_LIST << 30) | mask);
  }
}

// the coarse EMPTY bitmap over coarse_sc: one thread per 32-bit word
__global__ __launch_bounds__(256) void k_build_cmask(const uint32_t* __restrict__ coarse_sc, int gxc, int gyc, int shift,
                                                     int cw, int ch, int64_t nwords, uint32_t* __restrict__ out) {
  for (int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wi < nwords; wi += (int64_t)gridDim.x * blockDim.x) {
    uint32_t w = 0;
    for (int k = 0; k < 32; ++k) {
      const int64_t b = wi * 32 + k;
      if (b >= (int64_t)cw * ch) break;
      const int by = (int)(b / cw), bx = (int)(b % cw);
      bool empty = true;
      for (int y = by << shift; empty && y < min(gyc, (by + 1) << shift); ++y)
        for (int x = bx << shift; x < min(gxc, (bx + 1) << shift); ++x)
          if ((coarse_sc[(int64_t)y * gxc + x] >> 30) != CELL_EMPTY) { empty = false; break; }
      if (empty) w |= 1u << k;
    }
    out[wi] = w;
  }
}

// The row predicate's core rectangles (PipDev::core): for every polygon, a large rectangle of fine
// cells whose words are all INTERIOR(p).  Any such rectangle is exact (a row in it gets the answer its
// cell word gives).  The search runs on the coarse grid -- the largest rectangle of INTERIOR(p) coarse
// cells with its top-left corner on any cell, extents capped at CORE_CAP coarse cells so the build
// stays linear in the coarse grid -- and k_core_write widens it over the fine cells.
constexpr int CORE_CAP = 256;

// run[i] = how many coarse cells from i rightwards (<= CORE_CAP) carry i's INTERIOR word; 0 otherwise
__global__ __launch_bounds__(256) void k_core_run(const uint32_t* __restrict__ coarse_sc, int gxc, int64_t n,
                                                  int32_t n_polys, int32_t* __restrict__ run) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = coarse_sc[i];
    int r = 0;
    if ((w >> 30) == CELL_INTERIOR && (int64_t)(w & 0x3fffffffu) < n_polys) {
      const int xc = (int)(i % gxc);
      r = 1;
      while (r < CORE_CAP && xc + r < gxc && coarse_sc[i + r] == w) ++r;
    }
    run[i] = r;
  }
}

// the largest rectangle with its top-left corner on coarse cell i (first maximum scanning down)
__device__ __forceinline__ int core_rect(const uint32_t* coarse_sc, const int32_t* run, int gxc, int gyc, int64_t i,
                                         int& bw, int& bh) {
  const uint32_t w = coarse_sc[i];
  const int yc = (int)(i / gxc);
  int best = 0, wmin = run[i];
  bw = bh = 0;
  for (int h = 1; h <= CORE_CAP && yc + h - 1 < gyc && wmin > 0; ++h) {
    const int64_t j = i + (int64_t)(h - 1) * gxc;
    wmin = coarse_sc[j] == w ? min(wmin, (int)run[j]) : 0;
    if (wmin * h > best) { best = wmin * h; bw = wmin; bh = h; }
  }
  return best;
}

// best[p] = max over p's cells of (area << 40 | cell): deterministic (ties go to the larger cell index)
__global__ __launch_bounds__(256) void k_core_best(const uint32_t* __restrict__ coarse_sc, const int32_t* __restrict__ run,
                                                   int gxc, int gyc, unsigned long long* __restrict__ best) {
  const int64_t n = (int64_t)gxc * gyc;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (run[i] == 0) continue;
    int bw, bh;
    const int a = core_rect(coarse_sc, run, gxc, gyc, i, bw, bh);
    if (a > 0) atomicMax(&best[coarse_sc[i] & 0x3fffffffu], ((unsigned long long)a << 40) | (unsigned long long)i);
  }
}

// core[p] in fine cells: the coarse rectangle widened cell by cell (at most one coarse cell per side)
// while the new column / row of fine cells still carries INTERIOR(p) -- the fine cells of the mixed
// coarse ring around it that are interior too
__global__ __launch_bounds__(256) void k_core_write(const uint32_t* __restrict__ coarse_sc, const uint32_t* __restrict__ cell_sc,
                                                    const int32_t* __restrict__ run, int gx, int gy, int gxc, int gyc,
                                                    const unsigned long long* __restrict__ best, int32_t n_polys,
                                                    ushort4* __restrict__ core) {
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < n_polys; p += gridDim.x * blockDim.x) {
    const unsigned long long v = best[p];
    ushort4 r = make_ushort4(1, 1, 0, 0);   // none
    if (v) {
      const int64_t i = (int64_t)(v & ((1ull << 40) - 1));
      int bw, bh;
      core_rect(coarse_sc, run, gxc, gyc, i, bw, bh);
      const int xc = (int)(i % gxc), yc = (int)(i / gxc);
      const uint32_t w = coarse_sc[i];
      int X0 = xc << CF_LOG, Y0 = yc << CF_LOG;
      int X1 = min(gx, (xc + bw) << CF_LOG) - 1, Y1 = min(gy, (yc + bh) << CF_LOG) - 1;
      auto col_ok = [&](int X) {
        if (X < 0 || X >= gx) return false;
        for (int Y = Y0; Y <= Y1; ++Y)
          if (cell_sc[(int64_t)Y * gx + X] != w) return false;
        return true;
      };
      auto row_ok = [&](int Y) {
        if (Y < 0 || Y >= gy) return false;
        for (int X = X0; X <= X1; ++X)
          if (cell_sc[(int64_t)Y * gx + X] != w) return false;
        return true;
      };
      for (int k = 0; k < (1 << CF_LOG); ++k) {
        bool grew = false;
        if (col_ok(X0 - 1)) { --X0; grew = true; }
        if (col_ok(X1 + 1)) { ++X1; grew = true; }
        if (row_ok(Y0 - 1)) { --Y0; grew = true; }
        if (row_ok(Y1 + 1)) { ++Y1; grew = true; }
        if (!grew) break;
      }
      r = make_ushort4((unsigned short)X0, (unsigned short)Y0, (unsigned short)X1, (unsigned short)Y1);
    }
    core[p] = r;
  }
}

// pass 0 (ent == nullptr): cell_sc = resolved words, is_line[c] = 1 for line cells;
// pass 1: the line entries at their scanned slots, and the LINE words
template <bool LINES>
__global__ __launch_bounds__(256) void k_build_shortcut(PipDev d, int64_t ncell, uint32_t* __restrict__ cell_sc,
                                                        int32_t* __restrict__ is_line, const int64_t* __restrict__ slot,
                                                        uint4* __restrict__ ent) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x) {
    if (LINES && !is_line[c]) continue;
    const uint32_t w = d.cell_word[c];
    uint32_t word = w;
    uint4 e[2];
    const int k = analyze_cell(d, c, w, &word, e);
    if (!LINES) {
      cell_sc[c] = k == 1 ? word : w;
      is_line[c] = k == 2;
    } else if (k == 2) {
      ent[2 * slot[c]] = e[0];
      ent[2 * slot[c] + 1] = e[1];
      cell_sc[c] = (CELL_BOUNDARY << 30) | BLOB_COMPACT | SC_LINE | (uint32_t)slot[c];
    }
  }
}

__global__ void k_build_max(const int32_t* __restrict__ v, int64_t n, int* __restrict__ out) {
  int m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, v[i]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

__global__ void k_build_slot_poly(const int32_t* __restrict__ task_poly, const int64_t* __restrict__ task_slot,
                                  int ntask, int32_t* __restrict__ slot_poly) {
  const int task = blockIdx.x;
  if (task >= ntask) return;
  for (int64_t i = task_slot[task] + threadIdx.x; i < task_slot[task + 1]; i += blockDim.x) slot_poly[i] = task_poly[task];
}

}  // namespace gm

struct gm_pip_index {
  gm_ctx* ctx = nullptr;
  gm::PipDev dev{};
  std::vector<void*> allocs;
  int32_t n_polys = 0;
  int64_t n_entries = 0, n_boundary = 0, n_records = 0, n_slow = 0, n_cells = 0, blob_bytes = 0, n_compact = 0;
  int64_t max_bnd_per_cell = 0;   // most BOUNDARY (cell, polygon) entries of any cell: work items per point
  int64_t max_ent_per_cell = 0;   // most (cell, polygon) entries of any cell: pairs per point
  int64_t n_lines = 0;            // line shortcut entries (make_shortcut)
  const int32_t* list_poly = nullptr;   // polygon of each list_ent slot (the row-wise predicate's list search)
  const void* arr[GM_PIP_INDEX_ARRAYS] = {};   // the device arrays in gm_pip_index_layout order
  int64_t arr_bytes[GM_PIP_INDEX_ARRAYS] = {};
};

using namespace gm;

namespace {

// device array k of the index (gm_pip_index_layout order): rings, slab_off, slab_edges, cell_word,
// coarse_word, compact, list_ent, blob
template <class T>
int upload(gm_pip_index* ix, int k, const std::vector<T>& v, const T** out) {
  void* p = nullptr;
  const size_t bytes = v.size() * sizeof(T);
  GM_HIP(hipMalloc(&p, std::max<size_t>(bytes, 16)));
  ix->allocs.push_back(p);
  ix->arr[k] = p;
  ix->arr_bytes[k] = (int64_t)bytes;
  *out = (const T*)p;
  return v.empty() ? GM_OK : copy_h2d(ix->ctx, p, v.data(), bytes);
}

// the row-wise predicate's polygon per list slot (derived on the device)
int make_list_poly(gm_pip_index* ix) {
  const int64_t ns = ix->arr_bytes[6] / 4;
  void* lp = nullptr;
  GM_HIP(hipMalloc(&lp, (size_t)std::max<int64_t>(ns, 4) * 4));
  ix->allocs.push_back(lp);
  ix->list_poly = (const int32_t*)lp;
  if (ns > 0) {
    hipLaunchKernelGGL(k_list_poly, dim3((unsigned)((ns + RTPB - 1) / RTPB)), dim3(RTPB), 0, ix->ctx->stream, ix->dev, ns,
                       (int32_t*)lp);
    GM_CHECK_LAUNCH();
  }
  return GM_OK;
}

// the shortcut tables of a built or imported index (device-derived, not part of the exported layout)
int make_shortcut(gm_pip_index* ix) {
  const int64_t ncell = ix->arr_bytes[3] / 4;
  hipStream_t s = ix->ctx->stream;
  void* p = nullptr;
  GM_HIP(hipMalloc(&p, (size_t)std::max<int64_t>(ncell, 1) * 4));
  ix->allocs.push_back(p);
  ix->dev.cell_sc = (const uint32_t*)p;
  ix->dev.line_ent = nullptr;
  ix->n_lines = 0;
  ix->dev.fault = nullptr;   // set per call (the call's scratch word)
  ix->dev.cm = nullptr;      // the coarse EMPTY bitmaps, built after coarse_sc
  ix->dev.cm_words = 0;
  ix->dev.cm2 = nullptr;
  ix->dev.cm2_words = 0;
  ix->dev.core = nullptr;    // the row predicate's core rectangles, built after the bitmaps
  ix->dev.n_core = 0;
  ix->dev.n_line = 0;
  ix->dev.n_compact_lines = ix->arr_bytes[5] / 128;
  ix->dev.n_blob16 = ix->arr_bytes[7] / 16;
  ix->dev.n_list = ix->arr_bytes[6] / 4;
  ix->dev.coarse_fmt = ix->n_polys < (1 << 14) ? COARSE_MAIN : COARSE_EMPTY_MASK;
  if (const char* f = getenv("GM_PIP_COARSE_FMT")) ix->dev.coarse_fmt = atoi(f) ? COARSE_MAIN : COARSE_EMPTY_MASK;   // tests
  if (ix->n_polys >= (1 << 14)) ix->dev.coarse_fmt = COARSE_EMPTY_MASK;   // main ids need 14 bits
  {   // the join's coarse table: EMPTY until k_build_coarse_sc fills it
    const int64_t nh = std::max<int64_t>(1, (int64_t)ix->dev.gxc * ((ix->dev.gy + (1 << CF_LOG) - 1) >> CF_LOG));
    void* cp = nullptr;
    GM_HIP(hipMalloc(&cp, (size_t)nh * 4));
    ix->allocs.push_back(cp);
    ix->dev.coarse_sc = (const uint32_t*)cp;
    GM_HIP(hipMemsetD32Async((hipDeviceptr_t)cp, CELL_EMPTY << 30, (size_t)nh, s));
  }
  if (ncell == 0) return GM_OK;
  const bool lines_ok = ix->arr_bytes[5] / 128 < (int64_t)SC_LINE;   // compact indices below the LINE bit
  void *fl = nullptr, *sl = nullptr, *part = nullptr;
  auto cleanup = [&]() { (void)hipFree(fl); (void)hipFree(sl); (void)hipFree(part); };
  if (hipMalloc(&fl, (size_t)ncell * 4) != hipSuccess || hipMalloc(&sl, (size_t)(ncell + 1) * 8) != hipSuccess ||
      hipMalloc(&part, (size_t)scan_partials_len(ncell) * 8) != hipSuccess) {
    cleanup();
    return hip_fail(hipErrorOutOfMemory, "gm_pip_index shortcut");
  }
  const unsigned g = (unsigned)std::min<int64_t>(65536, (ncell + 255) / 256);
  hipLaunchKernelGGL(k_build_shortcut<false>, dim3(g), dim3(256), 0, s, ix->dev, ncell, (uint32_t*)p, (int32_t*)fl,
                     nullptr, nullptr);
  launch_excl_scan(s, (const int32_t*)fl, ncell, (int64_t*)sl, (int64_t*)part, (int64_t*)sl + ncell);
  int64_t nl = 0;
  int rc = copy_d2h(ix->ctx, &nl, (int64_t*)sl + ncell, 8);
  if (!rc && nl > 0 && lines_ok && nl < (int64_t)SC_LINE) {
    void* e = nullptr;
    if (hipMalloc(&e, (size_t)nl * 2 * sizeof(uint4)) != hipSuccess) { cleanup(); return hip_fail(hipErrorOutOfMemory, "gm_pip_index lines"); }
    ix->allocs.push_back(e);
    ix->dev.line_ent = (const uint4*)e;
    ix->n_lines = nl;
    ix->dev.n_line = nl;
    hipLaunchKernelGGL(k_build_shortcut<true>, dim3(g), dim3(256), 0, s, ix->dev, ncell, (uint32_t*)p, (int32_t*)fl,
                       (const int64_t*)sl, (uint4*)e);
  }
  if (!rc) {
    const int gxc = ix->dev.gxc, gyc = (ix->dev.gy + (1 << CF_LOG) - 1) >> CF_LOG;
    hipLaunchKernelGGL(k_build_coarse_sc, dim3((unsigned)std::min<int64_t>(65536, ((int64_t)gxc * gyc + 255) / 256)), dim3(256),
                       0, s, (const uint32_t*)p, ix->dev.gx, ix->dev.gy, gxc, gyc, ix->dev.coarse_fmt,
                       (uint32_t*)ix->dev.coarse_sc);
    // the coarse EMPTY bitmaps: the finest block size whose bitmap fits each kernel's LDS budget
    // (the join's, the row predicate's)
    auto bitmap = [&](int64_t budget_words, const uint32_t** out, int32_t* shift, int32_t* w, int64_t* words) -> int {
      int sh = 0;
      while ((int64_t)((gxc + (1 << sh) - 1) >> sh) * ((gyc + (1 << sh) - 1) >> sh) > budget_words * 32) ++sh;
      const int cw = (gxc + (1 << sh) - 1) >> sh, ch = (gyc + (1 << sh) - 1) >> sh;
      const int64_t nw = ((int64_t)cw * ch + 31) / 32;
      void* cm = nullptr;
      if (hipMalloc(&cm, (size_t)nw * 4) != hipSuccess) return hip_fail(hipErrorOutOfMemory, "gm_pip_index bitmap");
      ix->allocs.push_back(cm);
      hipLaunchKernelGGL(k_build_cmask, dim3((unsigned)std::min<int64_t>(4096, (nw + 255) / 256)), dim3(256), 0, s,
                         (const uint32_t*)ix->dev.coarse_sc, gxc, gyc, sh, cw, ch, nw, (uint32_t*)cm);
      *out = (const uint32_t*)cm; *shift = sh; *w = cw; *words = nw;
      return GM_OK;
    };
    rc = bitmap(CM_WORDS_MAX, &ix->dev.cm, &ix->dev.cm_shift, &ix->dev.cm_w, &ix->dev.cm_words);
    if (!rc) rc = bitmap(RELATE_CM_WORDS, &ix->dev.cm2, &ix->dev.cm2_shift, &ix->dev.cm2_w, &ix->dev.cm2_words);
    // the row predicate's core rectangles (fine-cell coordinates in 16 bits; polygon count within its LDS table)
    if (!rc && ix->n_polys > 0 && ix->n_polys <= RELATE_CORE_MAX && ix->dev.gx < 65535 && ix->dev.gy < 65535 &&
        !getenv("GM_PIP_NO_CORE")) {
      const int64_t nc = (int64_t)gxc * gyc;
      void *run = nullptr, *best = nullptr, *core = nullptr;
      if (hipMalloc(&run, (size_t)nc * 4) != hipSuccess || hipMalloc(&best, (size_t)ix->n_polys * 8) != hipSuccess ||
          hipMalloc(&core, (size_t)ix->n_polys * 8) != hipSuccess) {
        (void)hipFree(run); (void)hipFree(best); (void)hipFree(core);
        cleanup();
        return hip_fail(hipErrorOutOfMemory, "gm_pip_index core");
      }
      ix->allocs.push_back(core);
      const unsigned gc = (unsigned)std::min<int64_t>(65536, (nc + 255) / 256);
      hipLaunchKernelGGL(k_core_run, dim3(gc), dim3(256), 0, s, ix->dev.coarse_sc, gxc, nc, ix->n_polys, (int32_t*)run);
      GM_HIP(hipMemsetAsync(best, 0, (size_t)ix->n_polys * 8, s));
      hipLaunchKernelGGL(k_core_best, dim3(gc), dim3(256), 0, s, ix->dev.coarse_sc, (const int32_t*)run, gxc, gyc,
                         (unsigned long long*)best);
      hipLaunchKernelGGL(k_core_write, dim3((unsigned)((ix->n_polys + 255) / 256)), dim3(256), 0, s, ix->dev.coarse_sc,
                         ix->dev.cell_sc, (const int32_t*)run, ix->dev.gx, ix->dev.gy, gxc, gyc,
                         (const unsigned long long*)best, ix->n_polys, (ushort4*)core);
      const bool ok = hipStreamSynchronize(s) == hipSuccess;
      (void)hipFree(run); (void)hipFree(best);
      if (!ok) { cleanup(); return hip_fail(hipErrorLaunchFailure, "k_core_*"); }
      ix->dev.core = (const ushort4*)core;
      ix->dev.n_core = ix->n_polys;
    }
    if (rc) { cleanup(); return rc; }
  }
  if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "k_build_shortcut");
  cleanup();
  if (!rc && getenv("GM_PIP_DEBUG")) {   // coverage (diagnostic copies)
    std::vector<uint32_t> cw((size_t)ncell), sc((size_t)ncell);
    GM_HIP(hipMemcpy(cw.data(), ix->dev.cell_word, (size_t)ncell * 4, hipMemcpyDeviceToHost));
    GM_HIP(hipMemcpy(sc.data(), p, (size_t)ncell * 4, hipMemcpyDeviceToHost));
    int64_t nb = 0, nc = 0, nu = 0, ns = 0;
    for (int64_t c = 0; c < ncell; ++c) {
      if ((cw[(size_t)c] >> 30) != CELL_BOUNDARY) continue;
      ++nb;
      nc += (cw[(size_t)c] & BLOB_COMPACT) != 0;
      nu += (sc[(size_t)c] >> 30) != CELL_BOUNDARY;
      ns += (sc[(size_t)c] & (BLOB_COMPACT | SC_LINE)) == (BLOB_COMPACT | SC_LINE) && (sc[(size_t)c] >> 30) == CELL_BOUNDARY;
    }
    fprintf(stderr, "[gm_pip] shortcut: %lld boundary cell words (%lld compact), %lld uncrossed (one location), "
            "%lld line shortcuts\n", (long long)nb, (long long)nc, (long long)nu, (long long)ns);
  }
  return rc;
}

struct BandSeg {
  int32_t seg;   // global vertex id of the segment end (segment = v[seg-1] -> v[seg])
  double minx, maxx, ymin, ymax;
  int32_t vmin, vmax;  // vertex ids holding ymin / ymax
};

// breakpoints of a cell: y values of right-of-cell segment end points inside (yb0, yb1], ascending, unique
void collect_breakpoints(const std::vector<const BandSeg*>& right, double yb0, double yb1,
                         std::vector<std::pair<double, int32_t>>& bk) {
  bk.clear();
  for (const BandSeg* sg : right) {
    if (sg->ymin > yb0 && sg->ymin <= yb1) bk.push_back({sg->ymin, sg->vmin});
    if (sg->ymax > yb0 && sg->ymax <= yb1) bk.push_back({sg->ymax, sg->vmax});
  }
  std::sort(bk.begin(), bk.end(),
            [](const std::pair<double, int32_t>& x, const std::pair<double, int32_t>& y) { return x.first < y.first; });
  bk.erase(std::unique(bk.begin(), bk.end(),
                       [](const std::pair<double, int32_t>& x, const std::pair<double, int32_t>& y) {
                         return x.first == y.first;
                       }),
           bk.end());
}

// parity of right-of-cell segments straddling y (ymin <= y < ymax) at each breakpoint interval's left end
uint64_t right_parity(const std::vector<const BandSeg*>& right, double yb0,
                      const std::vector<std::pair<double, int32_t>>& bk) {
  uint64_t parity = 0;
  for (size_t j = 0; j <= bk.size(); ++j) {
    const double yk = j == 0 ? yb0 : bk[j - 1].first;
    int c = 0;
    for (const BandSeg* sg : right) c += (sg->ymin <= yk && yk < sg->ymax);
    if (c & 1) parity |= 1ull << j;
  }
  return parity;
}

// host threads of the index build: GM_BUILD_THREADS, else OMP_NUM_THREADS (16 on the GPU boxes),
// else the machine's, at most 64
int build_threads() {
  for (const char* v : {"GM_BUILD_THREADS", "OMP_NUM_THREADS"}) {
    const char* s = getenv(v);
    if (s && atoi(s) > 0) return std::min(64, atoi(s));
  }
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(64u, hc ? hc : 1u));
}

// fn(i) for i in [0, n) over the build threads (contiguous blocks of items per thread)
template <class F>
void parallel_for(int n, F fn) {
  const int nth = std::max(1, std::min(build_threads(), n / 64));
  if (nth <= 1) { for (int i = 0; i < n; ++i) fn(i); return; }
  std::atomic<int> next{0};
  auto work = [&]() {
    for (;;) {
      const int b = next.fetch_add(64);
      if (b >= n) break;
      for (int i = b; i < std::min(n, b + 64); ++i) fn(i);
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nth; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Device build of the cell words, coarse words, lists and blobs (k_build_rows and friends); the
// rings / slab arrays stay host-built.  Returns GM_OK, an error, or 1 = "not handled here" (the
// caller then runs the host classification).  Fills ix arrays 3-7 and the counters.
int build_cells_device(gm_ctx* ctx, gm_pip_index* ix, const gm_polyset* ps, const std::vector<double>& env,
                       const double* G, double inv_cw, double inv_ch, double epsx, double epsy, int gx, int gy,
                       const RingDev* d_rings) {
  hipStream_t s = ctx->stream;
  const int P = ps->n_polys;
  const int n_parts = P ? ps->poly_part_off[P] : 0;
  const int n_rings = n_parts ? ps->part_ring_off[n_parts] : 0;
  const int n_verts = n_rings ? ps->ring_vert_off[n_rings] : 0;
  // tasks = (polygon, row); slots = cells of a task's row
  std::vector<int32_t> task_poly, task_cy;
  std::vector<int64_t> task_slot{0}, band_off;
  int64_t band_total = 0;
  for (int p = 0; p < P; ++p) {
    const double* e = &env[4 * (size_t)p];
    if (!(e[0] <= e[2])) continue;
    int nr = 0, ne = 0;
    for (int q = ps->poly_part_off[p]; q < ps->poly_part_off[p + 1]; ++q)
      for (int r = ps->part_ring_off[q]; r < ps->part_ring_off[q + 1]; ++r) {
        ++nr;
        ne += std::max(0, ps->ring_vert_off[r + 1] - ps->ring_vert_off[r] - 1);
      }
    if (nr > BUILD_MAXR) return 1;
    const int cx0 = host::cell_of(e[0], G[0], inv_cw, gx), cx1 = host::cell_of(e[2], G[0], inv_cw, gx);
    const int cy0 = host::cell_of(e[1], G[1], inv_ch, gy), cy1 = host::cell_of(e[3], G[1], inv_ch, gy);
    for (int cy = cy0; cy <= cy1; ++cy) {
      task_poly.push_back(p);
      task_cy.push_back(cy);
      task_slot.push_back(task_slot.back() + (cx1 - cx0 + 1));
      if (ne > BAND_LDS) { band_off.push_back(band_total); band_total += ne; }
      else band_off.push_back(-1);
    }
  }
  const int64_t ntask = (int64_t)task_poly.size(), nslot = task_slot.back();
  if (ntask == 0 || ntask > INT32_MAX) return 1;
  // very large rings spanning many rows would need a huge global band scratch (a slice of the
  // polygon's edge count per row task): those sets are left to the host build
  if (band_total > ((int64_t)1 << 27)) return 1;
  const int64_t ncell = (int64_t)gx * gy;
  std::vector<void*> tmp;
  auto dalloc = [&](size_t bytes, void** p) -> int {
    GM_HIP(hipMalloc(p, std::max<size_t>(bytes, 16)));
    tmp.push_back(*p);
    return GM_OK;
  };
  auto cleanup = [&]() { for (void* p : tmp) (void)hipFree(p); tmp.clear(); };
  auto up = [&](const void* h, size_t bytes, void** d) -> int {
    int rc = dalloc(bytes, d);
    if (!rc && bytes) rc = copy_h2d(ctx, *d, h, bytes);
    return rc;
  };
  BuildArgs a{};
  int rc = GM_OK;
  void *d_ppo, *d_pro, *d_rvo, *d_vx, *d_vy, *d_env, *d_tp, *d_tc, *d_ts, *d_bo;
  rc = up(ps->poly_part_off, (size_t)(P + 1) * 4, &d_ppo);
  if (!rc) rc = up(ps->part_ring_off, (size_t)(n_parts + 1) * 4, &d_pro);
  if (!rc) rc = up(ps->ring_vert_off, (size_t)(n_rings + 1) * 4, &d_rvo);
  if (!rc) rc = up(ps->vx, (size_t)n_verts * 8, &d_vx);
  if (!rc) rc = up(ps->vy, (size_t)n_verts * 8, &d_vy);
  if (!rc) rc = up(env.data(), env.size() * 8, &d_env);
  if (!rc) rc = up(task_poly.data(), (size_t)ntask * 4, &d_tp);
  if (!rc) rc = up(task_cy.data(), (size_t)ntask * 4, &d_tc);
  if (!rc) rc = up(task_slot.data(), (size_t)(ntask + 1) * 8, &d_ts);
  if (!rc) rc = up(band_off.data(), (size_t)ntask * 8, &d_bo);
  void *d_bseg = nullptr, *d_bring = nullptr, *d_bmnx = nullptr, *d_bmxx = nullptr, *d_bmny = nullptr, *d_bmxy = nullptr;
  if (!rc) rc = dalloc((size_t)band_total * 4, &d_bseg);
  if (!rc) rc = dalloc((size_t)band_total * 4, &d_bring);
  if (!rc) rc = dalloc((size_t)band_total * 8, &d_bmnx);
  if (!rc) rc = dalloc((size_t)band_total * 8, &d_bmxx);
  if (!rc) rc = dalloc((size_t)band_total * 8, &d_bmny);
  if (!rc) rc = dalloc((size_t)band_total * 8, &d_bmxy);
  void *d_gw, *d_cl, *d_goff, *d_coff, *d_part, *d_stat;
  const int64_t np = scan_partials_len(nslot);
  if (!rc) rc = dalloc((size_t)nslot * 4, &d_gw);
  if (!rc) rc = dalloc((size_t)nslot * 4, &d_cl);
  if (!rc) rc = dalloc((size_t)(nslot + 1) * 8, &d_goff);
  if (!rc) rc = dalloc((size_t)(nslot + 1) * 8, &d_coff);
  if (!rc) rc = dalloc((size_t)std::max(np, scan_partials_len(ncell)) * 8, &d_part);
  if (!rc) rc = dalloc(8 * 8, &d_stat);
  if (rc) { cleanup(); return rc; }
  GM_HIP(hipMemsetAsync(d_stat, 0, 64, s));
  a.poly_part_off = (const int32_t*)d_ppo; a.part_ring_off = (const int32_t*)d_pro;
  a.ring_vert_off = (const int32_t*)d_rvo; a.vx = (const double*)d_vx; a.vy = (const double*)d_vy;
  a.rings = d_rings; a.env = (const double*)d_env;
  a.task_poly = (const int32_t*)d_tp; a.task_cy = (const int32_t*)d_tc; a.task_slot = (const int64_t*)d_ts;
  a.band_off = (const int64_t*)d_bo;
  a.band_g = BandView{(int32_t*)d_bseg, (int32_t*)d_bring, (double*)d_bmnx, (double*)d_bmxx, (double*)d_bmny,
                      (double*)d_bmxy};
  a.G0 = G[0]; a.G1 = G[1]; a.inv_cw = inv_cw; a.inv_ch = inv_ch; a.epsx = epsx; a.epsy = epsy;
  a.gx = gx; a.gy = gy;
  a.gen_words = (int32_t*)d_gw; a.cmp_lines = (int32_t*)d_cl;
  a.stat = (unsigned long long*)d_stat;
  // count pass -> slot offsets
  a.write = 0;
  hipLaunchKernelGGL(k_build_rows, dim3((unsigned)ntask), dim3(BT_TPB), 0, s, a);
  GM_CHECK_LAUNCH();
  launch_excl_scan(s, (const int32_t*)d_gw, nslot, (int64_t*)d_goff, (int64_t*)d_part, (int64_t*)d_goff + nslot);
  launch_excl_scan(s, (const int32_t*)d_cl, nslot, (int64_t*)d_coff, (int64_t*)d_part, (int64_t*)d_coff + nslot);
  GM_CHECK_LAUNCH();
  int64_t tot_words = 0, tot_lines = 0;
  unsigned long long st[4];
  rc = copy_d2h(ctx, &tot_words, (int64_t*)d_goff + nslot, 8);
  if (!rc) rc = copy_d2h(ctx, &tot_lines, (int64_t*)d_coff + nslot, 8);
  if (!rc) rc = copy_d2h(ctx, st, d_stat, sizeof st);
  if (rc) { cleanup(); return rc; }
  if (tot_words / 2 >= (int64_t)BLOB_COMPACT || tot_lines >= (int64_t)BLOB_COMPACT) {
    cleanup();
    gm::set_error("gm_pip_index_create: boundary blobs too large (lower cells_per_poly)");
    return GM_E_CAPACITY;
  }
  // the index arrays this build produces
  void *d_blob, *d_cmp, *d_cw, *d_coarse, *d_list;
  const int64_t blob_words = std::max<int64_t>(tot_words, 1), cmp_words = std::max<int64_t>(tot_lines, 1) * 16;
  auto own = [&](int k, size_t bytes, void** p) -> int {
    GM_HIP(hipMalloc(p, std::max<size_t>(bytes, 16)));
    ix->allocs.push_back(*p);
    ix->arr[k] = *p;
    ix->arr_bytes[k] = (int64_t)bytes;
    return GM_OK;
  };
  rc = own(7, (size_t)blob_words * 8, &d_blob);
  if (!rc) rc = own(5, (size_t)cmp_words * 8, &d_cmp);
  if (!rc) rc = own(3, (size_t)ncell * 4, &d_cw);
  if (rc) { cleanup(); return rc; }
  GM_HIP(hipMemsetAsync(d_blob, 0, (size_t)blob_words * 8, s));
  GM_HIP(hipMemsetAsync(d_cmp, 0, (size_t)cmp_words * 8, s));
  void *d_ew, *d_ec;
  rc = dalloc((size_t)nslot * 4, &d_ew);
  if (!rc) rc = dalloc((size_t)nslot * 4, &d_ec);
  if (rc) { cleanup(); return rc; }
  a.write = 1;
  a.gen_off = (const int64_t*)d_goff; a.cmp_off = (const int64_t*)d_coff;
  a.ent_word = (uint32_t*)d_ew; a.ent_cell = (int32_t*)d_ec;
  a.blob = (double*)d_blob; a.compact = (double*)d_cmp;
  hipLaunchKernelGGL(k_build_rows, dim3((unsigned)ntask), dim3(BT_TPB), 0, s, a);
  GM_CHECK_LAUNCH();
  // entries per cell -> buckets -> cell words and lists
  void *d_pc, *d_bc, *d_cs, *d_fill, *d_sp, *d_ll, *d_lo, *d_max;
  rc = dalloc((size_t)ncell * 4, &d_pc);
  if (!rc) rc = dalloc((size_t)ncell * 4, &d_bc);
  if (!rc) rc = dalloc((size_t)(ncell + 1) * 8, &d_cs);
  if (!rc) rc = dalloc((size_t)ncell * 4, &d_fill);
  if (!rc) rc = dalloc((size_t)nslot * 4, &d_sp);
  if (!rc) rc = dalloc((size_t)ncell * 4, &d_ll);
  if (!rc) rc = dalloc((size_t)(ncell + 1) * 8, &d_lo);
  if (!rc) rc = dalloc(16, &d_max);
  if (rc) { cleanup(); return rc; }
  GM_HIP(hipMemsetAsync(d_pc, 0, (size_t)ncell * 4, s));
  GM_HIP(hipMemsetAsync(d_bc, 0, (size_t)ncell * 4, s));
  GM_HIP(hipMemsetAsync(d_fill, 0, (size_t)ncell * 4, s));
  GM_HIP(hipMemsetAsync(d_max, 0, 16, s));
  const unsigned g1 = (unsigned)std::min<int64_t>(65536, (std::max(nslot, ncell) + 255) / 256);
  hipLaunchKernelGGL(k_build_cell_count, dim3(g1), dim3(256), 0, s, (const uint32_t*)d_ew, (const int32_t*)d_ec, nslot,
                     (int32_t*)d_pc, (int32_t*)d_bc);
  launch_excl_scan(s, (const int32_t*)d_pc, ncell, (int64_t*)d_cs, (int64_t*)d_part, (int64_t*)d_cs + ncell);
  hipLaunchKernelGGL(k_build_slot_poly, dim3((unsigned)ntask), dim3(256), 0, s, (const int32_t*)d_tp,
                     (const int64_t*)d_ts, (int)ntask, (int32_t*)d_sp);
  GM_CHECK_LAUNCH();
  int64_t n_ent = 0;
  rc = copy_d2h(ctx, &n_ent, (int64_t*)d_cs + ncell, 8);
  if (rc) { cleanup(); return rc; }
  void* d_bucket;
  rc = dalloc((size_t)std::max<int64_t>(n_ent, 1) * 8, &d_bucket);
  if (rc) { cleanup(); return rc; }
  hipLaunchKernelGGL(k_build_cell_scatter, dim3(g1), dim3(256), 0, s, (const uint32_t*)d_ew, (const int32_t*)d_ec, nslot,
                     (const int64_t*)d_cs, (int32_t*)d_fill, (uint32_t*)d_bucket, (const int32_t*)d_sp);
  hipLaunchKernelGGL(k_build_list_len, dim3(g1), dim3(256), 0, s, (const int32_t*)d_pc, ncell, (int32_t*)d_ll);
  launch_excl_scan(s, (const int32_t*)d_ll, ncell, (int64_t*)d_lo, (int64_t*)d_part, (int64_t*)d_lo + ncell);
  GM_CHECK_LAUNCH();
  int64_t n_list = 0;
  rc = copy_d2h(ctx, &n_list, (int64_t*)d_lo + ncell, 8);
  if (rc) { cleanup(); return rc; }
  if (n_list / 4 + 1 >= ((int64_t)1 << 26)) {
    cleanup();
    gm::set_error("gm_pip_index_create: cell lists too large");
    return GM_E_CAPACITY;
  }
  const int64_t list_slots = std::max<int64_t>(n_list, 4);
  rc = own(6, (size_t)list_slots * 4, &d_list);
  if (rc) { cleanup(); return rc; }
  GM_HIP(hipMemsetAsync(d_list, 0, (size_t)list_slots * 4, s));
  hipLaunchKernelGGL(k_build_cells, dim3(g1), dim3(256), 0, s, (const int32_t*)d_pc, (const int64_t*)d_cs,
                     (uint32_t*)d_bucket, (const int64_t*)d_lo, ncell, (uint32_t*)d_cw, (uint32_t*)d_list);
  GM_CHECK_LAUNCH();
  const int gxc = (gx + (1 << CF_LOG) - 1) >> CF_LOG, gyc = (gy + (1 << CF_LOG) - 1) >> CF_LOG;
  rc = own(4, (size_t)gxc * gyc * 4, &d_coarse);
  if (rc) { cleanup(); return rc; }
  hipLaunchKernelGGL(k_build_coarse, dim3((unsigned)std::min<int64_t>(65536, ((int64_t)gxc * gyc + 255) / 256)),
                     dim3(256), 0, s, (const uint32_t*)d_cw, gx, gy, gxc, gyc, (uint32_t*)d_coarse);
  hipLaunchKernelGGL(k_build_max, dim3(g1), dim3(256), 0, s, (const int32_t*)d_pc, ncell, (int*)d_max);
  hipLaunchKernelGGL(k_build_max, dim3(g1), dim3(256), 0, s, (const int32_t*)d_bc, ncell, (int*)d_max + 1);
  GM_CHECK_LAUNCH();
  int mx[2] = {0, 0};
  rc = copy_d2h(ctx, mx, d_max, 8);
  cleanup();
  if (rc) return rc;
  ix->dev.cell_word = (const uint32_t*)d_cw;
  ix->dev.coarse_word = (const uint32_t*)d_coarse;
  ix->dev.compact = (const double*)d_cmp;
  ix->dev.list_ent = (const uint32_t*)d_list;
  ix->dev.blob = (const double*)d_blob;
  ix->dev.gxc = gxc;
  ix->max_ent_per_cell = mx[0];
  ix->max_bnd_per_cell = mx[1];
  ix->n_entries = n_ent;
  ix->n_slow = (int64_t)st[0];
  ix->n_records = (int64_t)st[1];
  ix->n_boundary = (int64_t)st[2];
  ix->n_compact = (int64_t)st[3];
  ix->blob_bytes = (std::max<int64_t>(tot_words, 1) + tot_lines * 16) * 8;   // the host build pads an empty blob array to one word
  return GM_OK;
}

}  // namespace

// persistent grid: exactly the resident block count of this kernel (a rounded multiple of 8 for
// the XCD-aware mapping), so no partial second round of blocks forms a tail
// a reference check of the join failed on the device (PIP_FAULT_* bits): nothing of the call's
// output is trusted
static int index_fault(const char* what, uint32_t bits) {
  char msg[160];
  snprintf(msg, sizeof msg, "%s: device reference check failed (PIP_FAULT bits 0x%x): corrupt index or internal "
           "queue invariant", what, bits);
  set_error(msg);
  return GM_E_INDEX;
}

template <class K>
static unsigned resident_grid(K kernel, int device, int64_t ntiles, bool xcd_multiple) {
  const int resident = resident_blocks((const void*)kernel, device, JTPB, 4);
  int64_t g = std::min<int64_t>(resident, std::max<int64_t>(ntiles, 1));
  if (xcd_multiple) g = (g + 7) / 8 * 8;
  return (unsigned)g;
}

// rows per join pass: the strategy's limit, lowered by the context's GM_PARAM_JOIN_CHUNK
static int64_t join_chunk(const gm_ctx* ctx, int64_t limit) {
  return ctx->join_chunk > 0 ? std::min<int64_t>(limit, ctx->join_chunk) : limit;
}

template <bool WRITE, bool REC, bool SPLIT, int SRC = 0>
static unsigned join_grid(int device, int64_t ntiles) {
  return resident_grid(k_pip_join<WRITE, REC, SPLIT, SRC>, device, ntiles, REC);
}

// the staged direct pass (k_pip_join_q) over rows [0, m) of one chunk; GM_PIP_JOIN_LEGACY=1 selects
// the round-2 single-stage kernel (k_pip_join) for A/B measurement
static bool join_legacy() {
  const char* e = getenv("GM_PIP_JOIN_LEGACY");
  return e && atoi(e) != 0;
}

// The staged direct pass over n rows in chunks of at most 2^31 (32-bit row ids in the queues).  With
// outputs, each chunk's waves write slabs, then k_pair_plan / k_pair_move close the holes, so
// [0, counter[0]) is contiguous before the next chunk reserves past it.  SRC / VEC as k_pip_join_q;
// `ap` is the Arrow column (tuple bytes `tb`) when SRC != 0.
template <int SRC, bool VEC>
static int join_staged(gm_ctx* ctx, const double* px, const double* py, ArrowPts ap, size_t tb, int64_t n,
                       int64_t id_base, const PipDev& dv, int64_t* pt_ids, int32_t* poly_ids, int64_t cap,
                       unsigned long long* counter) {
  const bool write = pt_ids && poly_ids;
  const int64_t CHUNK = join_chunk(ctx, (int64_t)1 << 31);
  const int resident = write ? resident_blocks((const void*)k_pip_join_q<true, SRC, VEC>, ctx->device, QTPB, 1)
                             : resident_blocks((const void*)k_pip_join_q<false, SRC, VEC>, ctx->device, QTPB, 1);
  const int64_t wmax = (int64_t)resident * (QTPB / 64);
  if (write && wmax > PLAN_MAX) return hip_fail(hipErrorInvalidValue, "join: more waves than the pair plan holds");
  PairOut po{pt_ids, poly_ids, cap, nullptr, nullptr, 0, counter, nullptr};
  PairPlan* plan = nullptr;
  if (write) {   // context workspace: overflow ids | overflow polygons | wave descriptors | plan
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const int64_t ocap = wmax * SLAB;
    const size_t a_id = al((size_t)ocap * 8), a_pl = al((size_t)ocap * 4), a_d = al((size_t)wmax * sizeof(longlong2));
    void* base = nullptr;
    int rc = ctx_workspace(ctx, WS_JOIN, a_id + a_pl + a_d + sizeof(PairPlan), &base);
    if (rc) return rc;
    char* q = (char*)base;
    po.opt = (int64_t*)q; q += a_id;
    po.opl = (int32_t*)q; q += a_pl;
    po.desc = (longlong2*)q; q += a_d;
    po.ocap = ocap;
    plan = (PairPlan*)q;
  }
  for (int64_t c0 = 0; c0 < n; c0 += CHUNK) {
    const int64_t m = std::min(CHUNK, n - c0);
    const int64_t wsteps = ((m + 1) / 2 + 63) / 64;   // 128-point stream steps, one wave each
    const int64_t blocks = (wsteps + QTPB / 64 - 1) / (QTPB / 64);
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(resident, blocks));
    ArrowPts a = ap;
    if (SRC != 0) { a.c = (const char*)ap.c + (size_t)c0 * tb; a.voff = ap.voff + c0; }
    const double* cx = SRC == 0 ? px + c0 : nullptr;
    const double* cy = SRC == 0 ? py + c0 : nullptr;
    if (write) {
      hipLaunchKernelGGL((k_pip_join_q<true, SRC, VEC>), dim3(grid), dim3(QTPB), 0, ctx->stream, cx, cy, m, id_base + c0,
                         dv, po, (int64_t)0, a);
      hipLaunchKernelGGL(k_pair_plan, dim3(1), dim3(1024), 0, ctx->stream, (const longlong2*)po.desc,
                         (int)(grid * (QTPB / 64)), counter, plan);
      hipLaunchKernelGGL(k_pair_move, dim3(1024), dim3(256), 0, ctx->stream, po, (const PairPlan*)plan);
    } else {
      hipLaunchKernelGGL((k_pip_join_q<false, SRC, VEC>), dim3(grid), dim3(QTPB), 0, ctx->stream, cx, cy, m,
                         id_base + c0, dv, po, (int64_t)0, a);
    }
    GM_CHECK_LAUNCH();
  }
  return GM_OK;
}

// the direct pass over an Arrow point column (tuples read in place)
template <int SRC>
static int join_direct_arrow(gm_ctx* ctx, const gm_pip_index* ix, ArrowPts ap, int64_t n, int64_t id_base,
                             int64_t* pt_ids, int32_t* poly_ids, int64_t cap, unsigned long long* counter, int32_t op) {
  PipDev dv = ix->dev;
  dv.op = op;
  dv.fault = (uint32_t*)(counter + 1);
  const bool write = pt_ids && poly_ids;
  const int64_t CHUNK = join_chunk(ctx, (int64_t)1 << 31);
  const size_t tb = SRC == 2 ? 8 : 16;
  for (int64_t c0 = 0; c0 < n; c0 += CHUNK) {
    const int64_t m = std::min(CHUNK, n - c0);
    const int64_t ntiles = (m + JTILE - 1) / JTILE;
    ArrowPts a = ap;
    a.c = (const char*)ap.c + (size_t)c0 * tb;
    a.voff = ap.voff + c0;
    if (!join_legacy()) {
      if (c0 == 0) {
        const int rc = join_staged<SRC, false>(ctx, nullptr, nullptr, ap, tb, n, id_base, dv, pt_ids, poly_ids, cap, counter);
        if (rc) return rc;
      }
      continue;
    } else if (write)
      hipLaunchKernelGGL((k_pip_join<true, false, false, SRC>), dim3(join_grid<true, false, false, SRC>(ctx->device, ntiles)),
                         dim3(JTPB), 0, ctx->stream, nullptr, nullptr, nullptr, nullptr, m, id_base + c0, dv,
                         pt_ids, poly_ids, cap, counter, SplitArgs{}, a);
    else
      hipLaunchKernelGGL((k_pip_join<false, false, false, SRC>), dim3(join_grid<false, false, false, SRC>(ctx->device, ntiles)),
                         dim3(JTPB), 0, ctx->stream, nullptr, nullptr, nullptr, nullptr, m, id_base + c0, dv,
                         pt_ids, poly_ids, cap, counter, SplitArgs{}, a);
    GM_CHECK_LAUNCH();
  }
  return GM_OK;
}

extern "C" {

int gm_pip_index_create(gm_ctx* ctx, const gm_polyset* ps, gm_pip_index** out) {
  return gm_pip_index_create_ex(ctx, ps, 0, out);
}

int gm_pip_index_create_ex(gm_ctx* ctx, const gm_polyset* ps, int cells_per_poly_in, gm_pip_index** out) {
  if (!ctx || !ps || !out || ps->n_polys < 0 || cells_per_poly_in < 0) return GM_E_INVALID;
  *out = nullptr;
  const double t_start = now_s();
  const int P = ps->n_polys;
  if (P > 0 && (!ps->poly_part_off || !ps->part_ring_off || !ps->ring_vert_off)) return GM_E_INVALID;
  const int n_parts = P ? ps->poly_part_off[P] : 0;
  const int n_rings = n_parts ? ps->part_ring_off[n_parts] : 0;
  const int n_verts = n_rings ? ps->ring_vert_off[n_rings] : 0;
  if (n_verts > 0 && (!ps->vx || !ps->vy)) return GM_E_INVALID;
  const double* vx = ps->vx;
  const double* vy = ps->vy;

  // ---- rings: envelopes + y-slab segment buckets (fallback walk); segments by end vertex
  std::vector<RingDev> rings((size_t)n_rings);
  std::vector<int32_t> slab_off;
  std::vector<Edge> slab_edges, segs((size_t)std::max(n_verts, 1));  // segs: segment ending at vertex i
  // per ring: envelope and slab count (parallel over rings), then flat counting-sort of the
  // segments into their slabs (two passes over each ring, no per-slab vectors)
  std::vector<int64_t> ring_slab_base((size_t)n_rings + 1, 0), ring_edge_base((size_t)n_rings + 1, 0);
  {
    auto ring_env = [&](int r) {
      const int v0 = ps->ring_vert_off[r], v1 = ps->ring_vert_off[r + 1];
      RingDev& rd = rings[r];
      rd.minx = rd.miny = INFINITY;
      rd.maxx = rd.maxy = -INFINITY;
      for (int v = v0; v < v1; ++v) {
        rd.minx = std::min(rd.minx, vx[v]); rd.maxx = std::max(rd.maxx, vx[v]);
        rd.miny = std::min(rd.miny, vy[v]); rd.maxy = std::max(rd.maxy, vy[v]);
      }
      for (int i = v0 + 1; i < v1; ++i) segs[i] = Edge{vx[i], vy[i], vx[i - 1], vy[i - 1]};
      const int nseg = std::max(0, v1 - v0 - 1);
      int ns = std::max(1, std::min(4096, nseg / 2));
      const double hgt = rd.maxy - rd.miny;
      if (!(hgt > 0.0) || nseg == 0) ns = 1;
      rd.y0 = nseg ? rd.miny : 0.0;
      rd.inv_h = (ns > 1) ? (double)ns / hgt : 0.0;
      rd.ns = ns;
      int64_t ne = 0;   // (segment, slab) pairs of the ring
      for (int i = v0 + 1; i < v1; ++i) {
        const int s0 = host::cell_of(std::min(vy[i], vy[i - 1]), rd.y0, rd.inv_h, ns);
        const int s1 = host::cell_of(std::max(vy[i], vy[i - 1]), rd.y0, rd.inv_h, ns);
        ne += s1 - s0 + 1;
      }
      ring_edge_base[r + 1] = ne;
      ring_slab_base[r + 1] = ns;
    };
    parallel_for(n_rings, ring_env);
    for (int r = 0; r < n_rings; ++r) {
      ring_slab_base[r + 1] += ring_slab_base[r];
      ring_edge_base[r + 1] += ring_edge_base[r];
      rings[r].slab_base = (int32_t)ring_slab_base[r];
    }
    slab_off.assign((size_t)ring_slab_base[n_rings] + 1, 0);
    slab_edges.resize((size_t)ring_edge_base[n_rings]);
    auto ring_fill = [&](int r) {
      const int v0 = ps->ring_vert_off[r], v1 = ps->ring_vert_off[r + 1];
      const RingDev& rd = rings[r];
      const int ns = rd.ns;
      int32_t* so = slab_off.data() + ring_slab_base[r];
      std::vector<int32_t> cnt((size_t)ns + 1, 0);
      for (int i = v0 + 1; i < v1; ++i) {
        const int s0 = host::cell_of(std::min(vy[i], vy[i - 1]), rd.y0, rd.inv_h, ns);
        const int s1 = host::cell_of(std::max(vy[i], vy[i - 1]), rd.y0, rd.inv_h, ns);
        for (int k = s0; k <= s1; ++k) cnt[k + 1]++;
      }
      for (int k = 0; k < ns; ++k) cnt[k + 1] += cnt[k];
      for (int k = 0; k < ns; ++k) so[k] = (int32_t)(ring_edge_base[r] + cnt[k]);
      Edge* out = slab_edges.data() + ring_edge_base[r];
      for (int i = v0 + 1; i < v1; ++i) {   // segments in vertex order within each slab
        const int s0 = host::cell_of(std::min(vy[i], vy[i - 1]), rd.y0, rd.inv_h, ns);
        const int s1 = host::cell_of(std::max(vy[i], vy[i - 1]), rd.y0, rd.inv_h, ns);
        for (int k = s0; k <= s1; ++k) out[cnt[k]++] = segs[i];
      }
    };
    parallel_for(n_rings, ring_fill);
    slab_off[(size_t)ring_slab_base[n_rings]] = (int32_t)slab_edges.size();
  }

  // ---- polygon envelopes (JTS: Polygon envelope = shell envelope; MultiPolygon = union)
  std::vector<double> env((size_t)std::max(P, 1) * 4);
  double G[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
  for (int p = 0; p < P; ++p) {
    double e[4] = {INFINITY, INFINITY, -INFINITY, -INFINITY};
    for (int q = ps->poly_part_off[p]; q < ps->poly_part_off[p + 1]; ++q) {
      const int r0 = ps->part_ring_off[q];
      if (ps->part_ring_off[q + 1] <= r0) continue;
      const RingDev& rd = rings[r0];
      e[0] = std::min(e[0], rd.minx); e[1] = std::min(e[1], rd.miny);
      e[2] = std::max(e[2], rd.maxx); e[3] = std::max(e[3], rd.maxy);
    }
    memcpy(&env[4 * (size_t)p], e, sizeof e);
    if (e[0] <= e[2]) {
      G[0] = std::min(G[0], e[0]); G[1] = std::min(G[1], e[1]);
      G[2] = std::max(G[2], e[2]); G[3] = std::max(G[3], e[3]);
    }
  }
  const bool any = G[0] <= G[2];
  if (!any) { G[0] = G[1] = 0.0; G[2] = G[3] = -1.0; }  // nothing can match

  // ---- grid: ~cells_per_poly cells per polygon over the set's envelope
  const double W = any ? G[2] - G[0] : 0.0, H = any ? G[3] - G[1] : 0.0;
  const int64_t cells_per_poly = cells_per_poly_in > 0 ? cells_per_poly_in : 8192;
  int64_t target = std::min<int64_t>(std::max<int64_t>((int64_t)P * cells_per_poly, 64), (int64_t)1 << GM_MAX_CELLS_LOG);
  int gx = 1, gy = 1;
  const bool degenerate = !(W > 0 && H > 0);
  if (!degenerate) {
    gx = (int)std::max<double>(1.0, std::floor(std::sqrt((double)target * W / H)));
    gy = (int)std::max<int64_t>(1, target / gx);
  }
  const double inv_cw = degenerate ? 0.0 : (double)gx / W, inv_ch = degenerate ? 0.0 : (double)gy / H;
  const double epsx = W > 0 ? W * 1e-9 : 1e-9, epsy = H > 0 ? H * 1e-9 : 1e-9;
  const int64_t ncell = (int64_t)gx * gy;

  // ---- device build (default): cell words, lists and blobs built on the GPU from the polygon CSR
  if (!degenerate && any && ctx->index_build == 0) {
    gm_pip_index* ix = new gm_pip_index();
    ix->ctx = ctx;
    int rc = GM_OK;
    GM_HIP(hipSetDevice(ctx->device));
    rc = upload(ix, 0, rings, &ix->dev.rings);
    if (!rc) rc = upload(ix, 1, slab_off, &ix->dev.slab_off);
    if (!rc) rc = upload(ix, 2, slab_edges, &ix->dev.slab_edges);
    const double t_prep = now_s();
    if (!rc) rc = build_cells_device(ctx, ix, ps, env, G, inv_cw, inv_ch, epsx, epsy, gx, gy, ix->dev.rings);
    if (rc == 1) {
      gm_pip_index_destroy(ix);   // not handled on the device: the host classification below
    } else if (rc) {
      gm_pip_index_destroy(ix);
      return rc;
    } else {
      ix->n_polys = P;
      ix->n_cells = ncell;
      ix->dev.gx0 = G[0]; ix->dev.gy0 = G[1]; ix->dev.gx1 = G[2]; ix->dev.gy1 = G[3];
      ix->dev.inv_cw = inv_cw; ix->dev.inv_ch = inv_ch;
      ix->dev.gx = gx; ix->dev.gy = gy;
      rc = make_list_poly(ix);
      if (!rc) rc = make_shortcut(ix);
      if (rc) { gm_pip_index_destroy(ix); return rc; }
      if (getenv("GM_PIP_DEBUG")) {
        GM_HIP(hipStreamSynchronize(ctx->stream));
        fprintf(stderr, "[gm_pip] device build: rings + slabs %.3f s, cells %.3f s; %lld cells, %lld entries, "
                "%lld blob bytes\n", t_prep - t_start, now_s() - t_prep, (long long)ncell, (long long)ix->n_entries,
                (long long)ix->blob_bytes);
      }
      *out = ix;
      return GM_OK;
    }
  }

  // ---- (cell, polygon) classification + boundary blobs, in parallel over chunks of polygons.  A
  // chunk's entries carry chunk-local blob / compact offsets; the chunks are concatenated in polygon
  // order afterwards (so cell lists keep polygons ascending) and the offsets rebased.
  struct Ent { int64_t cell; uint32_t e; };
  struct ChunkOut {
    std::vector<Ent> ents;
    std::vector<double> blob;      // 8-byte words; each blob starts 16-byte aligned (even length kept)
    std::vector<double> compact;   // 16-word (128-B) compact blobs
    int64_t n_slow = 0, n_boundary = 0, n_records = 0, n_compact = 0;
  };
  constexpr int PCH = 4;   // polygons per work item
  const int nchunks = (P + PCH - 1) / PCH;
  std::vector<ChunkOut> outs((size_t)std::max(nchunks, 1));
  std::atomic<int> next_chunk{0};
  struct RingRef { int32_t ring; bool shell; };
  auto classify = [&]() {
    std::vector<RingRef> ring_list;
    std::vector<std::vector<BandSeg>> band;  // per ring of the polygon, segments meeting the row band
    std::vector<int32_t> a_edges;
    std::vector<const BandSeg*> right;
    std::vector<std::pair<double, int32_t>> bk;
    for (;;) {
      const int ch = next_chunk.fetch_add(1);
      if (ch >= nchunks || !any) break;
      ChunkOut& o = outs[(size_t)ch];
      std::vector<Ent>& ents = o.ents;
      std::vector<double>& blob = o.blob;
      std::vector<double>& compact = o.compact;
      auto put_i32x2 = [&](int32_t a, int32_t b) {
        double w; int32_t v[2] = {a, b}; memcpy(&w, v, 8); blob.push_back(w);
      };
      auto put_u64 = [&](uint64_t u) { double w; memcpy(&w, &u, 8); blob.push_back(w); };
      for (int p = ch * PCH; p < std::min(P, (ch + 1) * PCH); ++p) {
        const double* e = &env[4 * (size_t)p];
        if (!(e[0] <= e[2])) continue;
        ring_list.clear();
        for (int q = ps->poly_part_off[p]; q < ps->poly_part_off[p + 1]; ++q)
          for (int r = ps->part_ring_off[q]; r < ps->part_ring_off[q + 1]; ++r)
            ring_list.push_back(RingRef{r, r == ps->part_ring_off[q]});
        const int nr = (int)ring_list.size();
        band.resize((size_t)nr);
        const int cx0 = host::cell_of(e[0], G[0], inv_cw, gx), cx1 = host::cell_of(e[2], G[0], inv_cw, gx);
        const int cy0 = host::cell_of(e[1], G[1], inv_ch, gy), cy1 = host::cell_of(e[3], G[1], inv_ch, gy);
        for (int cy = cy0; cy <= cy1; ++cy) {
          const double yb0 = degenerate ? -INFINITY : G[1] + (double)cy / inv_ch - epsy;
          const double yb1 = degenerate ? INFINITY : G[1] + (double)(cy + 1) / inv_ch + epsy;
          for (int k = 0; k < nr; ++k) {
            band[k].clear();
            const int r = ring_list[k].ring;
            for (int i = ps->ring_vert_off[r] + 1; i < ps->ring_vert_off[r + 1]; ++i) {
              const double ya = vy[i - 1], yb = vy[i];
              const double ymin = std::min(ya, yb), ymax = std::max(ya, yb);
              if (ymax < yb0 || ymin > yb1) continue;
              band[k].push_back(BandSeg{i, std::min(vx[i - 1], vx[i]), std::max(vx[i - 1], vx[i]), ymin, ymax,
                                        ya <= yb ? i - 1 : i, ya <= yb ? i : i - 1});
            }
          }
          int run_loc = -1;
          for (int cx = cx0; cx <= cx1; ++cx) {
            const int64_t cell = (int64_t)cy * gx + cx;
            const double xb0 = degenerate ? -INFINITY : G[0] + (double)cx / inv_cw - epsx;
            const double xb1 = degenerate ? INFINITY : G[0] + (double)(cx + 1) / inv_cw + epsx;
            bool bnd = degenerate;
            for (int k = 0; k < nr && !bnd; ++k)
              for (const BandSeg& sg : band[k])
                if (sg.maxx >= xb0 && sg.minx <= xb1) { bnd = true; break; }
            if (!bnd) {
              if (run_loc < 0) {
                // any point of the cell: its nominal centre, checked to map back to the cell
                const double cxm = G[0] + ((double)cx + 0.5) / inv_cw;
                const double cym = G[1] + ((double)cy + 0.5) / inv_ch;
                if (host::cell_of(cxm, G[0], inv_cw, gx) != cx || host::cell_of(cym, G[1], inv_ch, gy) != cy) bnd = true;
                else run_loc = host::locate_poly(ps, p, cxm, cym);
              }
              if (!bnd) {
                if (run_loc == LOC_EXTERIOR) continue;
                if (run_loc == LOC_INTERIOR) {
                  ents.push_back(Ent{cell, (CELL_INTERIOR << 30) | (uint32_t)p});
                  continue;
                }
                bnd = true;  // a boundary location cannot occur in a segment-free cell; stay exact anyway
              }
            }
            run_loc = -1;
            // ---- compact blob: single-ring polygon, <= 2 segments, <= 4 breakpoints -> one 128-B line
            if (nr == 1 && !degenerate) {
              a_edges.clear(); right.clear(); bk.clear();
              for (const BandSeg& sg : band[0]) {
                if (sg.maxx >= xb0 && sg.minx <= xb1) a_edges.push_back(sg.seg);
                else if (sg.minx > xb1) right.push_back(&sg);
              }
              collect_breakpoints(right, yb0, yb1, bk);
              if (4 * a_edges.size() + bk.size() <= 30) {
                const int E = (int)a_edges.size(), B = (int)bk.size();
                const int lines = (4 * E + B <= 14 && E <= 3) ? 1 : 2;
                const uint64_t ci = compact.size() / 16;   // chunk-local line index
                double rec[32];
                for (double& w : rec) w = INFINITY;
                { int32_t v[2] = {p, E | (lines << 8)}; memcpy(&rec[0], v, 8); }
                { const uint64_t par = right_parity(right, yb0, bk); memcpy(&rec[1], &par, 8); }
                bool used[32] = {};
                used[0] = used[1] = true;
                for (int j = 0; j < E; ++j) {
                  const int32_t i = a_edges[j];
                  double* eg = rec + cseg_word(j);
                  eg[0] = vx[i]; eg[1] = vy[i]; eg[2] = vx[i - 1]; eg[3] = vy[i - 1];
                  for (int q = 0; q < 4; ++q) used[cseg_word(j) + q] = true;
                }
                int w = 2;
                for (int j = 0; j < B; ++j) {
                  while (used[w]) ++w;
                  rec[w] = bk[j].first;
                  used[w] = true;
                }
                compact.insert(compact.end(), rec, rec + 16 * lines);
                o.n_boundary++;
                o.n_compact++;
                ents.push_back(Ent{cell, (CELL_BOUNDARY << 30) | BLOB_COMPACT | (uint32_t)ci});
                continue;
              }
            }
            // ---- boundary blob
            if (blob.size() & 1) blob.push_back(0.0);
            const uint64_t boff = blob.size() / 2;   // chunk-local, 16-B units
            put_i32x2(p, nr);
            for (int k = 0; k < nr; ++k) {
              a_edges.clear(); right.clear(); bk.clear();
              for (const BandSeg& sg : band[k]) {
                if (sg.maxx >= xb0 && sg.minx <= xb1) a_edges.push_back(sg.seg);
                else if (sg.minx > xb1) right.push_back(&sg);
              }
              collect_breakpoints(right, yb0, yb1, bk);
              const int r = ring_list[k].ring;
              const bool slow = degenerate || a_edges.size() > 4096 || bk.size() > 63;
              RingHdr rh{};
              rh.flags = (int16_t)((ring_list[k].shell ? 1 : 0) | (slow ? 2 : 0));
              rh.n_edge = slow ? 0 : (int16_t)a_edges.size();
              rh.n_brk = slow ? 0 : (int16_t)bk.size();
              { double w; memcpy(&w, &rh, 8); blob.push_back(w); }
              uint64_t parity = 0;
              if (!slow) {
                parity = right_parity(right, yb0, bk);
              } else {
                o.n_slow++;
                parity = (uint32_t)r;
              }
              put_u64(parity);
              if (!slow) {
                for (int32_t i : a_edges) {
                  blob.push_back(vx[i]); blob.push_back(vy[i]); blob.push_back(vx[i - 1]); blob.push_back(vy[i - 1]);
                }
                for (auto& b : bk) blob.push_back(b.first);
              }
              o.n_records++;
            }
            o.n_boundary++;
            ents.push_back(Ent{cell, (CELL_BOUNDARY << 30) | (uint32_t)boff});
          }
        }
      }
      if (blob.size() & 1) blob.push_back(0.0);
    }
  };
  {
    const int nth = std::max(1, std::min(build_threads(), nchunks));
    std::vector<std::thread> th;
    for (int t = 1; t < nth; ++t) th.emplace_back(classify);
    classify();
    for (auto& t : th) t.join();
  }
  const double t_classify = now_s();
  // concatenate the chunks in polygon order, rebasing blob / compact offsets
  std::vector<Ent> ents;
  std::vector<double> blob, compact;
  int64_t n_slow = 0, n_boundary = 0, n_records = 0, n_compact = 0;
  {
    size_t ne = 0, nbw = 0, ncw = 0;
    for (const ChunkOut& o : outs) { ne += o.ents.size(); nbw += o.blob.size(); ncw += o.compact.size(); }
    if (nbw / 2 >= (size_t)BLOB_COMPACT || ncw / 16 >= (size_t)BLOB_COMPACT) {
      gm::set_error("gm_pip_index_create: boundary blobs too large (lower cells_per_poly)");
      return GM_E_CAPACITY;
    }
    ents.reserve(ne); blob.reserve(nbw); compact.reserve(ncw);
    for (ChunkOut& o : outs) {
      const uint32_t bb = (uint32_t)(blob.size() / 2), cb = (uint32_t)(compact.size() / 16);
      for (const Ent& en : o.ents) {
        uint32_t e = en.e;
        if ((e >> 30) == CELL_BOUNDARY) e += (e & BLOB_COMPACT) ? cb : bb;
        ents.push_back(Ent{en.cell, e});
      }
      blob.insert(blob.end(), o.blob.begin(), o.blob.end());
      compact.insert(compact.end(), o.compact.begin(), o.compact.end());
      n_slow += o.n_slow; n_boundary += o.n_boundary; n_records += o.n_records; n_compact += o.n_compact;
      std::vector<Ent>().swap(o.ents); std::vector<double>().swap(o.blob); std::vector<double>().swap(o.compact);
    }
  }
  std::vector<int32_t> per_cell((size_t)ncell, 0), bnd_cell((size_t)ncell, 0);
  for (const Ent& en : ents) {
    per_cell[en.cell]++;
    if ((en.e >> 30) == CELL_BOUNDARY) bnd_cell[en.cell]++;
  }
  const double t_merge = now_s();
  if (blob.empty()) blob.push_back(0.0);
  // ---- cell words: single entries inline, multi-entry cells through a list (polygons ascending)
  std::vector<uint32_t> cell_word((size_t)ncell, 0xffffffffu);
  std::vector<uint32_t> list_ent;
  {
    std::vector<int32_t> start((size_t)ncell + 1, 0);
    for (int64_t c = 0; c < ncell; ++c) start[c + 1] = start[c] + per_cell[c];
    std::vector<uint32_t> all(ents.size());
    std::vector<int32_t> fill(start.begin(), start.end() - 1);
    for (const Ent& en : ents) all[fill[en.cell]++] = en.e;
    for (int64_t c = 0; c < ncell; ++c) {
      const int k = per_cell[c];
      if (k == 1) cell_word[c] = all[start[c]];
      else if (k > 1) {
        // payload = (list offset / 4) << 4 | count (15 = long list: true count in the first slot);
        // lists start 16-B aligned so one uint4 load brings the first four slots
        while (list_ent.size() & 3) list_ent.push_back(0);
        const size_t off = list_ent.size() / 4;
        if (off + k + 1 >= ((size_t)1 << 26)) { gm::set_error("gm_pip_index_create: cell lists too large"); return GM_E_CAPACITY; }
        cell_word[c] = (CELL_LIST << 30) | (uint32_t)(off << 4) | (uint32_t)std::min(k, LIST_LONG);
        if (k >= LIST_LONG) list_ent.push_back((uint32_t)k);
        for (int j = 0; j < k; ++j) list_ent.push_back(all[start[c] + j]);
      }
    }
  }
  while (list_ent.size() < 4 || (list_ent.size() & 3)) list_ent.push_back(0);
  // coarse words: EMPTY when every fine cell is empty, the fine word when all fine cells carry the
  // same INTERIOR word, otherwise CELL_LIST ("read the fine word")
  const int gxc = (gx + (1 << CF_LOG) - 1) >> CF_LOG, gyc = (gy + (1 << CF_LOG) - 1) >> CF_LOG;
  std::vector<uint32_t> coarse_word((size_t)gxc * gyc, 0xffffffffu);
  for (int yc = 0; yc < gyc; ++yc)
    for (int xc = 0; xc < gxc; ++xc) {
      uint32_t w = 0xffffffffu;
      bool first = true, mixed = false;
      for (int yy = yc << CF_LOG; yy < std::min(gy, (yc + 1) << CF_LOG) && !mixed; ++yy)
        for (int xx = xc << CF_LOG; xx < std::min(gx, (xc + 1) << CF_LOG); ++xx) {
          const uint32_t f = cell_word[(size_t)yy * gx + xx];
          if (first) { w = f; first = false; }
          else if (f != w) { mixed = true; break; }
        }
      const uint32_t kind = w >> 30;
      coarse_word[(size_t)yc * gxc + xc] =
          (!mixed && (kind == CELL_EMPTY || kind == CELL_INTERIOR)) ? w : (CELL_LIST << 30);
    }

  gm_pip_index* ix = new gm_pip_index();
  ix->ctx = ctx;
  ix->max_bnd_per_cell = ncell ? *std::max_element(bnd_cell.begin(), bnd_cell.end()) : 0;
  ix->max_ent_per_cell = ncell ? *std::max_element(per_cell.begin(), per_cell.end()) : 0;
  ix->n_polys = P;
  ix->n_entries = (int64_t)ents.size();
  ix->n_boundary = n_boundary;
  ix->n_records = n_records;
  ix->n_slow = n_slow;
  ix->n_compact = n_compact;
  ix->n_cells = ncell;
  ix->blob_bytes = (int64_t)(blob.size() + compact.size()) * 8;
  int rc = GM_OK;
  GM_HIP(hipSetDevice(ctx->device));
  if (!rc) rc = upload(ix, 0, rings, &ix->dev.rings);
  if (!rc) rc = upload(ix, 1, slab_off, &ix->dev.slab_off);
  if (!rc) rc = upload(ix, 2, slab_edges, &ix->dev.slab_edges);
  if (!rc) rc = upload(ix, 3, cell_word, &ix->dev.cell_word);
  if (!rc) rc = upload(ix, 4, coarse_word, &ix->dev.coarse_word);
  if (compact.empty()) compact.assign(16, 0.0);
  if (!rc) rc = upload(ix, 5, compact, &ix->dev.compact);
  if (!rc) rc = upload(ix, 6, list_ent, &ix->dev.list_ent);
  if (!rc) rc = upload(ix, 7, blob, &ix->dev.blob);
  if (rc) { gm_pip_index_destroy(ix); return rc; }
  ix->dev.gx0 = G[0]; ix->dev.gy0 = G[1]; ix->dev.gx1 = G[2]; ix->dev.gy1 = G[3];
  ix->dev.inv_cw = inv_cw; ix->dev.inv_ch = inv_ch;
  ix->dev.gx = gx; ix->dev.gy = gy; ix->dev.gxc = gxc;
  rc = make_list_poly(ix);
  if (!rc) rc = make_shortcut(ix);
  if (rc) { gm_pip_index_destroy(ix); return rc; }
  if (getenv("GM_PIP_DEBUG")) {
    GM_HIP(hipStreamSynchronize(ctx->stream));
    fprintf(stderr, "[gm_pip] build: classify %.3f s (%d threads), merge %.3f s, cell words + upload %.3f s; "
            "%lld cells, %lld entries, %lld blob bytes\n", t_classify - t_start, build_threads(), t_merge - t_classify,
            now_s() - t_merge, (long long)ncell, (long long)ix->n_entries, (long long)ix->blob_bytes);
  }
  *out = ix;
  return GM_OK;
}

int gm_pip_index_destroy(gm_pip_index* ix) {
  if (!ix) return GM_OK;
  for (void* p : ix->allocs) (void)hipFree(p);
  delete ix;
  return GM_OK;
}

int gm_pip_index_export(const gm_pip_index* ix, gm_pip_index_layout* lay) {
  if (!ix || !lay) return GM_E_INVALID;
  memset(lay, 0, sizeof(*lay));
  for (int k = 0; k < GM_PIP_INDEX_ARRAYS; ++k) lay->bytes[k] = ix->arr_bytes[k];
  const PipDev& d = ix->dev;
  const double g[6] = {d.gx0, d.gy0, d.gx1, d.gy1, d.inv_cw, d.inv_ch};
  memcpy(lay->grid, g, sizeof g);
  lay->dims[0] = d.gx; lay->dims[1] = d.gy; lay->dims[2] = d.gxc; lay->dims[3] = ix->n_polys;
  const int64_t st[9] = {ix->n_cells, ix->n_entries, ix->n_boundary, ix->n_records, ix->n_slow, ix->blob_bytes,
                         ix->n_compact, ix->max_bnd_per_cell, ix->max_ent_per_cell};
  memcpy(lay->stats, st, sizeof st);
  lay->version = GM_PIP_LAYOUT_VERSION;
  return GM_OK;
}

int gm_pip_index_copy_array(gm_ctx* ctx, const gm_pip_index* ix, int k, void* dst) {
  if (!ctx || !ix || k < 0 || k >= GM_PIP_INDEX_ARRAYS || (!dst && ix->arr_bytes[k])) return GM_E_INVALID;
  if (ix->arr_bytes[k])
    GM_HIP(hipMemcpyAsync(dst, ix->arr[k], (size_t)ix->arr_bytes[k], hipMemcpyDeviceToDevice, ctx->stream));
  return GM_OK;
}

int gm_pip_index_import(gm_ctx* ctx, const gm_pip_index_layout* lay, void* const* arrays, gm_pip_index** out) {
  if (!ctx || !lay || !arrays || !out || lay->version != GM_PIP_LAYOUT_VERSION) return GM_E_INVALID;
  *out = nullptr;
  for (int k = 0; k < GM_PIP_INDEX_ARRAYS; ++k)
    if (lay->bytes[k] < 0 || (lay->bytes[k] && !arrays[k])) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  gm_pip_index* ix = new gm_pip_index();
  ix->ctx = ctx;
  const void** dst[GM_PIP_INDEX_ARRAYS] = {(const void**)&ix->dev.rings, (const void**)&ix->dev.slab_off,
                                           (const void**)&ix->dev.slab_edges, (const void**)&ix->dev.cell_word,
                                           (const void**)&ix->dev.coarse_word, (const void**)&ix->dev.compact,
                                           (const void**)&ix->dev.list_ent, (const void**)&ix->dev.blob};
  for (int k = 0; k < GM_PIP_INDEX_ARRAYS; ++k) {
    void* p = nullptr;
    if (hipMalloc(&p, (size_t)std::max<int64_t>(lay->bytes[k], 16)) != hipSuccess) {
      gm_pip_index_destroy(ix);
      return hip_fail(hipErrorOutOfMemory, "gm_pip_index_import");
    }
    ix->allocs.push_back(p);
    ix->arr[k] = p;
    ix->arr_bytes[k] = lay->bytes[k];
    *dst[k] = p;
    if (lay->bytes[k] &&
        hipMemcpyAsync(p, arrays[k], (size_t)lay->bytes[k], hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess) {
      gm_pip_index_destroy(ix);
      return hip_fail(hipErrorInvalidValue, "gm_pip_index_import copy");
    }
  }
  PipDev& d = ix->dev;
  d.gx0 = lay->grid[0]; d.gy0 = lay->grid[1]; d.gx1 = lay->grid[2]; d.gy1 = lay->grid[3];
  d.inv_cw = lay->grid[4]; d.inv_ch = lay->grid[5];
  d.gx = lay->dims[0]; d.gy = lay->dims[1]; d.gxc = lay->dims[2];
  ix->n_polys = lay->dims[3];
  ix->n_cells = lay->stats[0]; ix->n_entries = lay->stats[1]; ix->n_boundary = lay->stats[2];
  ix->n_records = lay->stats[3]; ix->n_slow = lay->stats[4]; ix->blob_bytes = lay->stats[5];
  ix->n_compact = lay->stats[6]; ix->max_bnd_per_cell = lay->stats[7]; ix->max_ent_per_cell = lay->stats[8];
  int rc = make_list_poly(ix);
  if (!rc) rc = make_shortcut(ix);
  if (!rc && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "gm_pip_index_import");
  if (rc) { gm_pip_index_destroy(ix); return rc; }
  *out = ix;
  return GM_OK;
}

int gm_pip_index_stats(const gm_pip_index* ix, int64_t* stats) {
  if (!ix || !stats) return GM_E_INVALID;
  stats[0] = ix->n_cells;
  stats[1] = ix->n_entries;
  stats[2] = ix->n_boundary;
  stats[3] = ix->n_records;
  stats[4] = ix->n_slow;
  stats[5] = ix->blob_bytes;
  stats[6] = ix->n_compact;
  return GM_OK;
}

int gm_pip_index_core(gm_ctx* ctx, const gm_pip_index* ix, uint16_t* rects, int32_t* n_core) {
  if (!ctx || !ix || !n_core) return GM_E_INVALID;
  *n_core = ix->dev.core ? ix->dev.n_core : 0;
  if (!rects || *n_core == 0) return GM_OK;
  GM_HIP(hipSetDevice(ctx->device));
  return copy_d2h(ctx, rects, ix->dev.core, (size_t)*n_core * 8);
}

int gm_pip_join(gm_ctx* ctx, const gm_pip_index* ix, const double* px, const double* py, int64_t n, int64_t id_base,
                int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs) {
  return gm_pip_join_ex(ctx, ix, px, py, n, id_base, pt_ids, poly_ids, cap, n_pairs, GM_JOIN_AUTO);
}

int gm_pip_join_ex(gm_ctx* ctx, const gm_pip_index* ix, const double* px, const double* py, int64_t n,
                   int64_t id_base, int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode) {
  return gm_pip_join_pred(ctx, ix, px, py, n, id_base, pt_ids, poly_ids, cap, n_pairs, mode, GM_SPATIAL_CONTAINS);
}

int gm_pip_join_pred(gm_ctx* ctx, const gm_pip_index* ix, const double* px, const double* py, int64_t n,
                     int64_t id_base, int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode,
                     int predicate) {
  if (!ctx || !ix || n < 0 || cap < 0) return GM_E_INVALID;
  if (predicate != GM_SPATIAL_CONTAINS && predicate != GM_SPATIAL_INTERSECTS) return GM_E_INVALID;
  PipDev dv = ix->dev;
  dv.op = predicate == GM_SPATIAL_INTERSECTS ? JOIN_INTERSECTS : JOIN_CONTAINS;
  if (mode != GM_JOIN_AUTO && mode != GM_JOIN_DIRECT && mode != GM_JOIN_PARTITIONED && mode != GM_JOIN_SPLIT)
    return GM_E_INVALID;
  const bool write = pt_ids && poly_ids;
  if ((pt_ids == nullptr) != (poly_ids == nullptr)) return GM_E_INVALID;
  if (n > 0 && (!px || !py)) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  unsigned long long* counter = (unsigned long long*)ctx->d_scratch;
  dv.fault = (uint32_t*)(counter + 1);   // reference-check bits (PIP_FAULT_*), read back with the pair count
  GM_HIP(hipMemsetAsync(counter, 0, 16, ctx->stream));
  // AUTO = DIRECT at every size: measured on MI355X (1B CONUS points x 3,200 polygons) the direct pass takes 20 ms,
  // against 23 ms for the split pass and 39 ms for partition + join; the others stay
  // selectable
  if ((mode == GM_JOIN_AUTO || mode == GM_JOIN_DIRECT) && n > 0) {
    const int64_t CHUNK = join_chunk(ctx, (int64_t)1 << 31);  // LDS staging keeps 32-bit row offsets
    const bool vec = aligned16(px) && aligned16(py);   // chunk starts stay 16-B aligned (CHUNK is even)
    for (int64_t c0 = 0; c0 < n; c0 += CHUNK) {
      const int64_t m = std::min(CHUNK, n - c0);
      const int64_t ntiles = (m + JTILE - 1) / JTILE;
      if (!join_legacy()) {
        if (c0 == 0) {
          const int rc = vec ? join_staged<0, true>(ctx, px, py, ArrowPts{}, 16, n, id_base, dv, pt_ids, poly_ids, cap, counter)
                             : join_staged<0, false>(ctx, px, py, ArrowPts{}, 16, n, id_base, dv, pt_ids, poly_ids, cap, counter);
          if (rc) return rc;
        }
        continue;
      }
      const unsigned grid = write ? join_grid<true, false, false>(ctx->device, ntiles)
                                  : join_grid<false, false, false>(ctx->device, ntiles);
      if (write)
        hipLaunchKernelGGL((k_pip_join<true, false, false>), dim3(grid), dim3(JTPB), 0, ctx->stream, px + c0, py + c0,
                           nullptr, nullptr, m, id_base + c0, dv, pt_ids, poly_ids, cap, counter, SplitArgs{}, ArrowPts{});
      else
        hipLaunchKernelGGL((k_pip_join<false, false, false>), dim3(grid), dim3(JTPB), 0, ctx->stream, px + c0, py + c0,
                           nullptr, nullptr, m, id_base + c0, dv, pt_ids, poly_ids, cap, counter, SplitArgs{}, ArrowPts{});
      GM_CHECK_LAUNCH();
    }
  } else if (mode == GM_JOIN_SPLIT && n > 0) {
    // split pass per chunk: lookups + interior pairs + work list -> blob evaluations -> pack the
    // pair regions.  Worst-case region sizes follow from the index (entries per cell); the chunk is
    // sized so that items + pairs fit a 6 GiB context workspace (and rows stay 32-bit).
#ifdef GM_JX_CAPS   // timing experiment only: unsafe small segment capacities
    const int64_t per_b = 1, per_e = 1;
#else
    const int64_t per_b = std::max<int64_t>(1, ix->max_bnd_per_cell);
    const int64_t per_e = std::max<int64_t>(1, ix->max_ent_per_cell);
#endif
    if (getenv("GM_PIP_DEBUG")) fprintf(stderr, "[gm_pip] split: per_b %lld per_e %lld\n", (long long)per_b, (long long)per_e);
#ifndef GM_JOIN_WS_GB
#define GM_JOIN_WS_GB 6
#endif
    const int64_t budget = (int64_t)GM_JOIN_WS_GB << 30;
    int64_t CHUNK = join_chunk(ctx, std::min<int64_t>((int64_t)1 << 31,
                                                      budget / ((per_b + (write ? per_e : 0)) * (int64_t)sizeof(uint2))));
    CHUNK = std::max<int64_t>(JTILE * 8, CHUNK / (JTILE * 8) * (JTILE * 8));
    const int64_t mmax = std::min(CHUNK, n);
    const int64_t ntiles_max = (mmax + JTILE - 1) / JTILE;
    const unsigned grid_a = write ? join_grid<true, false, true>(ctx->device, ntiles_max)
                                  : join_grid<false, false, true>(ctx->device, ntiles_max);
    SplitArgs sp{};
    sp.nseg = (int32_t)grid_a * (JTPB / 64);
    const int64_t seg_pts = (ntiles_max + grid_a - 1) / grid_a * (int64_t)(64 * JILP);   // points one wave sees
    sp.ipw = seg_pts * per_b;
    sp.ppw = write ? seg_pts * per_e : 0;
    {
      auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
      const size_t a_items = al((size_t)sp.nseg * sp.ipw * sizeof(uint2)), a_pairs = al((size_t)sp.nseg * sp.ppw * sizeof(uint2));
      const size_t a_cnt = al((size_t)sp.nseg * 4), a_off = al((size_t)(sp.nseg + 1) * 8);
      void* base = nullptr;
      int wrc = ctx_workspace(ctx, WS_JOIN, a_items + a_pairs + 2 * a_cnt + a_off, &base);
      if (wrc) return wrc;
      char* q = (char*)base;
      sp.items = (uint2*)q; q += a_items;
      sp.pairs = (uint2*)q; q += a_pairs;
      sp.item_cnt = (uint32_t*)q; q += a_cnt;
      sp.pair_cnt = (uint32_t*)q; q += a_cnt;
      sp.pair_off = (int64_t*)q;
    }
    for (int64_t c0 = 0; c0 < n; c0 += CHUNK) {
      const int64_t m = std::min(CHUNK, n - c0);
      // every segment is written (counts) by its wave; the grid stays grid_a for every chunk
      if (write)
        hipLaunchKernelGGL((k_pip_join<true, false, true>), dim3(grid_a), dim3(JTPB), 0, ctx->stream, px + c0, py + c0,
                           nullptr, nullptr, m, id_base + c0, dv, pt_ids, poly_ids, cap, counter, sp, ArrowPts{});
      else
        hipLaunchKernelGGL((k_pip_join<false, false, true>), dim3(grid_a), dim3(JTPB), 0, ctx->stream, px + c0,
                           py + c0, nullptr, nullptr, m, id_base + c0, dv, pt_ids, poly_ids, cap, counter, sp, ArrowPts{});
      GM_CHECK_LAUNCH();
      const unsigned bgrid = write ? resident_grid(k_pip_blobs<true>, ctx->device, sp.nseg, false)
                                   : resident_grid(k_pip_blobs<false>, ctx->device, sp.nseg, false);
      if (write)
        hipLaunchKernelGGL((k_pip_blobs<true>), dim3(bgrid), dim3(JTPB), 0, ctx->stream, px + c0, py + c0, dv,
                           counter, sp);
      else
        hipLaunchKernelGGL((k_pip_blobs<false>), dim3(bgrid), dim3(JTPB), 0, ctx->stream, px + c0, py + c0, dv,
                           counter, sp);
      GM_CHECK_LAUNCH();
      if (write) {
        hipLaunchKernelGGL(k_pip_scan_segs, dim3(1), dim3(1024), 0, ctx->stream, sp);
        hipLaunchKernelGGL(k_pip_compact, dim3(std::min<int32_t>(sp.nseg, 4096)), dim3(JTPB), 0, ctx->stream, sp, counter,
                           id_base + c0, pt_ids, poly_ids, cap);
        hipLaunchKernelGGL(k_pip_chunk_done, dim3(1), dim3(64), 0, ctx->stream, sp, counter);
        GM_CHECK_LAUNCH();
      }
    }
  } else if (n > 0) {
    const int64_t CHUNK = join_chunk(ctx, (int64_t)1 << 28);  // 6 GiB of band-sorted records per pass
    const int rows_per_band = (ix->dev.gy + NBAND - 1) / NBAND;
    const int nb = (ix->dev.gy + rows_per_band - 1) / rows_per_band;
    const int64_t mmax = std::min(CHUNK, n);
    // one resident wave of partition blocks (each walks a contiguous slice of the chunk)
    const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(resident_grid(k_band_scatter<true>, ctx->device, 1 << 20, false),
                                                                 (mmax + PTILE - 1) / PTILE));
    const int64_t hlen = (int64_t)nb * nblk;
    uint32_t* hist = nullptr;
    uint32_t* pcount = nullptr;
    int64_t* poff = nullptr;
    PtRec* rec = nullptr;
    {  // context-owned workspace: records | histogram | per-block pair counts | pair slots
      const size_t a_rec = (size_t)mmax * sizeof(PtRec), a_h = ((size_t)(hlen + 1) * 4 + 15) & ~(size_t)15;
      const size_t a_pc = ((size_t)nblk * 4 + 15) & ~(size_t)15;
      void* base = nullptr;
      int wrc = ctx_workspace(ctx, WS_JOIN, a_rec + a_h + a_pc + (size_t)nblk * 8, &base);
      if (wrc) return wrc;
      rec = (PtRec*)base;
      hist = (uint32_t*)((char*)base + a_rec);
      pcount = (uint32_t*)((char*)base + a_rec + a_h);
      poff = (int64_t*)((char*)base + a_rec + a_h + a_pc);
    }
    int rc = GM_OK;
    for (int64_t c0 = 0; c0 < n && rc == GM_OK; c0 += CHUNK) {
      const int64_t m = std::min(CHUNK, n - c0);
      const int64_t per = ((m + nblk - 1) / nblk + PTILE - 1) / PTILE * PTILE;
      const unsigned pgrid = (unsigned)((m + per - 1) / per);   // <= nblk
      hipLaunchKernelGGL(k_band_hist, dim3(pgrid), dim3(PTPB), 0, ctx->stream, px + c0, py + c0, m, per, dv,
                         rows_per_band, nb, hist, pcount);
      hipLaunchKernelGGL(k_band_scan, dim3(1), dim3(1024), 0, ctx->stream, hist, (int64_t)nb * pgrid, pcount, (int)pgrid,
                         poff, counter);
      if (write)
        hipLaunchKernelGGL(k_band_scatter<true>, dim3(pgrid), dim3(PTPB), 0, ctx->stream, px + c0, py + c0, m, per, dv,
                           rows_per_band, nb, hist, rec, poff, id_base + c0, pt_ids, poly_ids, cap);
      else
        hipLaunchKernelGGL(k_band_scatter<false>, dim3(pgrid), dim3(PTPB), 0, ctx->stream, px + c0, py + c0, m, per, dv,
                           rows_per_band, nb, hist, rec, poff, id_base + c0, pt_ids, poly_ids, cap);
      const uint32_t* n_rec = hist + (int64_t)nb * pgrid;
      const int64_t ntiles = (m + JTILE - 1) / JTILE;
      const unsigned grid = write ? join_grid<true, true, false>(ctx->device, ntiles)
                                  : join_grid<false, true, false>(ctx->device, ntiles);
      if (write)
        hipLaunchKernelGGL((k_pip_join<true, true, false>), dim3(grid), dim3(JTPB), 0, ctx->stream, nullptr, nullptr,
                           rec, n_rec, m, id_base + c0, dv, pt_ids, poly_ids, cap, counter, SplitArgs{}, ArrowPts{});
      else
        hipLaunchKernelGGL((k_pip_join<false, true, false>), dim3(grid), dim3(JTPB), 0, ctx->stream, nullptr, nullptr,
                           rec, n_rec, m, id_base + c0, dv, pt_ids, poly_ids, cap, counter, SplitArgs{}, ArrowPts{});
      if (hipGetLastError() != hipSuccess) rc = hip_fail(hipErrorLaunchFailure, "k_pip_join (partitioned)");
    }
    if (rc) return rc;
  }
  if (n_pairs) {
    GM_HIP(hipMemcpyAsync(ctx->h_pinned, counter, 16, hipMemcpyDeviceToHost, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    *n_pairs = ctx->h_pinned[0];
    if (ctx->h_pinned[1]) return index_fault("gm_pip_join", (uint32_t)ctx->h_pinned[1]);
    if (write && *n_pairs > cap) return GM_E_CAPACITY;
  }
  return GM_OK;
}

int gm_pip_join_arrow(gm_ctx* ctx, const gm_pip_index* ix, const gm_geom_column* pts, int64_t n, int64_t id_base,
                      int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode, int predicate) {
  if (!ctx || !ix || n < 0 || cap < 0 || !pts) return GM_E_INVALID;
  if (predicate != GM_SPATIAL_CONTAINS && predicate != GM_SPATIAL_INTERSECTS) return GM_E_INVALID;
  const int32_t op = predicate == GM_SPATIAL_INTERSECTS ? JOIN_INTERSECTS : JOIN_CONTAINS;
  if (pts->type != GM_GEOM_POINT || (pts->ordinal_bits != 64 && pts->ordinal_bits != 32)) return GM_E_INVALID;
  if (n > 0 && !pts->coords) return GM_E_INVALID;
  if ((pt_ids == nullptr) != (poly_ids == nullptr)) return GM_E_INVALID;
  if (mode != GM_JOIN_AUTO && mode != GM_JOIN_DIRECT && mode != GM_JOIN_PARTITIONED && mode != GM_JOIN_SPLIT)
    return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  const ArrowPts ap{pts->coords, pts->validity, pts->validity_offset, pts->flip_axis, pts->ordinal_bits == 32};
  if (mode == GM_JOIN_AUTO || mode == GM_JOIN_DIRECT) {
    unsigned long long* counter = (unsigned long long*)ctx->d_scratch;
    GM_HIP(hipMemsetAsync(counter, 0, 16, ctx->stream));
    int rc = n == 0 ? GM_OK
             : ap.f32 ? join_direct_arrow<2>(ctx, ix, ap, n, id_base, pt_ids, poly_ids, cap, counter, op)
                      : join_direct_arrow<1>(ctx, ix, ap, n, id_base, pt_ids, poly_ids, cap, counter, op);
    if (rc) return rc;
    GM_HIP(hipMemcpyAsync(ctx->h_pinned, counter, 16, hipMemcpyDeviceToHost, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->h_pinned[1]) return index_fault("gm_pip_join_arrow", (uint32_t)ctx->h_pinned[1]);
    const int64_t total = ctx->h_pinned[0];
    if (n_pairs) *n_pairs = total;
    return (pt_ids && total > cap) ? GM_E_CAPACITY : GM_OK;
  }
  // the other strategies run on x / y columns
  double* xy = nullptr;
  GM_HIP(hipMallocAsync((void**)&xy, (size_t)std::max<int64_t>(n, 1) * 16, ctx->stream));
  int rc = gm_arrow_points_to_columns(ctx, pts, n, xy, xy + n);
  if (!rc) rc = gm_pip_join_pred(ctx, ix, xy, xy + n, n, id_base, pt_ids, poly_ids, cap, n_pairs, mode, predicate);
  (void)hipFreeAsync(xy, ctx->stream);
  return rc;
}

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
  const PipDev d = spatial_op != GM_SPATIAL_NONE ? geoms->dev : PipDev{};
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
  if (n_match && ids && *n_match > ids_cap) return GM_E_CAPACITY;
  return GM_OK;
}

int gm_pip_join_census(gm_ctx* ctx, const gm_pip_index* ix, const double* px, const double* py, int64_t n,
                       int64_t* counters) {
  if (!ctx || !ix || n < 0 || !counters || (n > 0 && (!px || !py))) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  unsigned long long* d = (unsigned long long*)ctx->d_scratch;
  static_assert(JC_N <= 16, "census counters exceed the context scratch");
  GM_HIP(hipMemsetAsync(d, 0, JC_N * 8, ctx->stream));
  if (n > 0) {
    hipLaunchKernelGGL(k_pip_census, dim3((unsigned)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0, ctx->stream,
                       px, py, n, ix->dev, d);
    GM_CHECK_LAUNCH();
  }
  return copy_d2h(ctx, counters, d, JC_N * 8);
}

int gm_pip_relate(gm_ctx* ctx, const gm_pip_index* ix, const int32_t* poly, const double* px, const double* py,
                  int64_t n, uint8_t* loc) {
  if (!ctx || !ix || n < 0) return GM_E_INVALID;
  if (n == 0) return GM_OK;
  if (!poly || !px || !py || !loc) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  const bool vec = RILP == 2 && ((uintptr_t)px | (uintptr_t)py) % 16 == 0 && (uintptr_t)poly % 8 == 0 &&
                   (uintptr_t)loc % 2 == 0 && !getenv("GM_PIP_RELATE_SCALAR");
  auto* kern = vec ? k_pip_relate<RILP == 2> : k_pip_relate<false>;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(resident_blocks((const void*)kern, ctx->device, RTPB, 1),
                                                                          (n + RTPB * RILP - 1) / (RTPB * RILP)));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(RTPB), 0, ctx->stream, poly, px, py, n, ix->n_polys, ix->dev,
                     ix->list_poly, loc);
  GM_CHECK_LAUNCH();
  return GM_OK;
}

}  // extern "C"
