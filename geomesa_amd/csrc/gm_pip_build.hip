// gm_pip_build.hip -- building the polygon index of gm_pip.hpp: the grid, the (cell, polygon)
// classification with boundary blobs (on the device by default, on the host with
// GM_PARAM_INDEX_BUILD = 1: byte-identical arrays), the derived shortcut tables, and the index's
// export / import for shipping it to other GPUs.  Reference: the broadcast side of
// GeoMesaJoinRelation (GeoMesaJoinRelation.scala:41-91) and RelationUtils.grid (RelationUtils.scala:30-157).
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <thread>

#include "gm_arrow.hpp"
#include "gm_pip.hpp"
#include "gm_scan.hpp"

namespace gm {

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
__global__ __launch_bounds__(256) void k_build_cmask(const uint32_t* __restrict__ coarse_sc, int gxc, int gyc, int shx,
                                                     int shy, int cw, int ch, int64_t nwords, uint32_t* __restrict__ out) {
  for (int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; wi < nwords; wi += (int64_t)gridDim.x * blockDim.x) {
    uint32_t w = 0;
    for (int k = 0; k < 32; ++k) {
      const int64_t b = wi * 32 + k;
      if (b >= (int64_t)cw * ch) break;
      const int by = (int)(b / cw), bx = (int)(b % cw);
      bool empty = true;
      for (int y = by << shy; empty && y < min(gyc, (by + 1) << shy); ++y)
        for (int x = bx << shx; x < min(gxc, (bx + 1) << shx); ++x)
          if ((coarse_sc[(int64_t)y * gxc + x] >> 30) != CELL_EMPTY) { empty = false; break; }
      if (empty) w |= 1u << k;
    }
    out[wi] = w;
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

// cell_sc8 (gm_pip.hpp, "8-B fine words"): cell_sc zero-extended; a LINE word of a polygon below 2^14
// replaced by its entry's lines when they fit:
//  * one line: requantized to 2^-12 cell (A / 4, B / 4, C / 4) when the deviation from the exact line
//    (entry deviation SC_DEV / 4 plus the rounding, over the enlarged cell) stays a unit below SC8_T;
//  * two lines meeting inside the cell: their intersection and normal angles at 10 bits (tag 2)
__global__ __launch_bounds__(256) void k_build_sc8(const uint32_t* __restrict__ cell_sc, const uint4* __restrict__ line_ent,
                                                   int64_t n_line, int64_t ncell, uint2* __restrict__ out) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = cell_sc[c];
    uint2 o = make_uint2(w, 0u);
    if (line_ent && (w >> 30) == CELL_BOUNDARY && (w & (BLOB_COMPACT | SC_LINE)) == (BLOB_COMPACT | SC_LINE) &&
        (uint64_t)(w & (SC_LINE - 1)) < (uint64_t)n_line) {
      const uint64_t li = w & (SC_LINE - 1);
      const uint4 e0 = line_ent[2 * li], e1 = line_ent[2 * li + 1];
      const uint32_t nl = e1.y >> 24;
      if (nl == 1u && e0.y < (1u << 14)) {
        const double A = (double)(int16_t)(e0.z & 0xffffu) / 4.0, B = (double)(int16_t)(e0.z >> 16) / 4.0;
        const double C = (double)((int32_t)(e0.w << 8) >> 8) / 4.0;
        const double a = rint(A), b = rint(B), cc = rint(C);
        double dev = 0.0;
        for (int q = 0; q < 4; ++q) {
          const double uc = (q & 1) ? 1.01 : -0.01, vc = (q & 2) ? 1.01 : -0.01;
          dev = fmax(dev, fabs((a - A) * uc + (b - B) * vc - (cc - C)));
        }
        if (dev + SC_DEV / 4.0 <= SC8_T - 1.0 && fabs(a) <= 8191.0 && fabs(b) <= 8191.0 && fabs(cc) <= 32767.0) {
          const uint64_t v = (1ull << 62) | ((uint64_t)e0.y << 48) | ((uint64_t)((e0.w >> 24) & 15u) << 44) |
                             (((uint64_t)(int64_t)a & 0x3fffu) << 30) | (((uint64_t)(int64_t)b & 0x3fffu) << 16) |
                             ((uint64_t)(int64_t)cc & 0xffffu);
          o = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
        }
      }
      else if (nl == 2u && e0.y < (1u << 14)) {
        const double A1 = (double)(int16_t)(e0.z & 0xffffu), B1 = (double)(int16_t)(e0.z >> 16);
        const double C1 = (double)((int32_t)(e0.w << 8) >> 8);
        const double A2 = (double)(int16_t)(e1.x & 0xffffu), B2 = (double)(int16_t)(e1.x >> 16);
        const double C2 = (double)((int32_t)(e1.y << 8) >> 8);
        const double det = A1 * B2 - A2 * B1;   // exact: |products| < 2^29
        if (fabs(det) >= 1.0) {
          const double vu = (C1 * B2 - C2 * B1) / det, vv = (A1 * C2 - A2 * C1) / det;
          if (vu >= 0.0 && vu < 1.0 && vv >= 0.0 && vv < 1.0) {
            const double tp = 6.283185307179586;
            auto ang = [&](double a_, double b_) -> uint32_t {
              double q = rint(atan2(b_, a_) / tp * 1024.0);
              if (q < 0) q += 1024.0;
              return (uint32_t)q & 1023u;
            };
            const uint64_t v = (2ull << 62) | ((uint64_t)e0.y << 48) | ((uint64_t)((e0.w >> 24) & 255u) << 40) |
                               ((uint64_t)((uint32_t)floor(vu * 1024.0) & 1023u) << 30) |
                               ((uint64_t)((uint32_t)floor(vv * 1024.0) & 1023u) << 20) |
                               ((uint64_t)ang(A1, B1) << 10) | (uint64_t)ang(A2, B2);
            o = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
          }
        }
      }
    }
    out[c] = o;
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

// ------------------------------------------------------------------ the row predicate's list search
__device__ __forceinline__ int entry_poly(const PipDev& d, uint32_t e) {
  const uint32_t ref = e & 0x3fffffffu;
  if ((e >> 30) == CELL_INTERIOR) return (int)ref;
  if (!blob_ref_ok(d, ref)) return -1;
  if (ref & BLOB_COMPACT) return (int)__double_as_longlong(d.compact[16 * (uint64_t)(ref & (BLOB_COMPACT - 1))]);
  return ((const int2*)(d.blob + 2 * (uint64_t)ref))->x;
}

__global__ __launch_bounds__(RTPB) void k_list_poly(PipDev d, int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * RTPB + threadIdx.x;
  if (i < n) out[i] = entry_poly(d, d.list_ent[i]);   // count / padding slots read as INTERIOR: no load
}

}  // namespace gm

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
  {   // the join's 8-B fine words (k_build_sc8, after the line entries)
    void* p8 = nullptr;
    GM_HIP(hipMalloc(&p8, (size_t)std::max<int64_t>(ncell, 1) * 8));
    ix->allocs.push_back(p8);
    ix->dev.cell_sc8 = (const uint2*)p8;
    if (ncell == 0) GM_HIP(hipMemsetD32Async((hipDeviceptr_t)p8, CELL_EMPTY << 30, 2, s));
  }
  ix->dev.line_ent = nullptr;
  ix->n_lines = 0;
  ix->dev.fault = nullptr;   // set per call (the call's scratch word)
  ix->dev.cm = nullptr;      // the coarse EMPTY bitmaps, built after coarse_sc
  ix->dev.cm_words = 0;
  ix->dev.rm = nullptr;
  ix->dev.rm_words = 0;
  ix->dev.n_line = 0;
  ix->dev.n_compact_lines = ix->arr_bytes[5] / 128;
  ix->dev.n_blob16 = ix->arr_bytes[7] / 16;
  ix->dev.n_list = ix->arr_bytes[6] / 4;
  // GM_PARAM_INDEX_COARSE; main polygon ids need 14 bits
  const int64_t cf = ix->ctx->index_coarse;
  ix->dev.coarse_fmt = (cf < 0 ? ix->n_polys < (1 << 14) : cf == 1) ? COARSE_MAIN : COARSE_EMPTY_MASK;
  if (ix->n_polys >= (1 << 14)) ix->dev.coarse_fmt = COARSE_EMPTY_MASK;
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
    hipLaunchKernelGGL(k_build_sc8, dim3(g), dim3(256), 0, s, (const uint32_t*)p, ix->dev.line_ent, ix->dev.n_line, ncell,
                       (uint2*)ix->dev.cell_sc8);
    const int gxc = ix->dev.gxc, gyc = (ix->dev.gy + (1 << CF_LOG) - 1) >> CF_LOG;
    hipLaunchKernelGGL(k_build_coarse_sc, dim3((unsigned)std::min<int64_t>(65536, ((int64_t)gxc * gyc + 255) / 256)), dim3(256),
                       0, s, (const uint32_t*)p, ix->dev.gx, ix->dev.gy, gxc, gyc, ix->dev.coarse_fmt,
                       (uint32_t*)ix->dev.coarse_sc);
    // the coarse EMPTY bitmaps: the finest block size whose bitmap fits each kernel's LDS budget
    // (the join's, the row predicate's)
    auto bitmap = [&](int64_t budget_words, const uint32_t** out, int32_t* shift, int32_t* shift_y, int32_t* w,
                      int64_t* words) -> int {
      // blocks of 2^shx x 2^shy coarse cells, shx = shy or shy + 1: the finest that fits the budget
      int shx = 0, shy = 0;
      while ((int64_t)((gxc + (1 << shx) - 1) >> shx) * ((gyc + (1 << shy) - 1) >> shy) > budget_words * 32) {
        if (shx == shy) ++shx;
        else ++shy;
      }
      const int cw = (gxc + (1 << shx) - 1) >> shx, ch = (gyc + (1 << shy) - 1) >> shy;
      const int64_t nw = ((int64_t)cw * ch + 31) / 32;
      void* cm = nullptr;
      if (hipMalloc(&cm, (size_t)nw * 4) != hipSuccess) return hip_fail(hipErrorOutOfMemory, "gm_pip_index bitmap");
      ix->allocs.push_back(cm);
      hipLaunchKernelGGL(k_build_cmask, dim3((unsigned)std::min<int64_t>(4096, (nw + 255) / 256)), dim3(256), 0, s,
                         (const uint32_t*)ix->dev.coarse_sc, gxc, gyc, shx, shy, cw, ch, nw, (uint32_t*)cm);
      *out = (const uint32_t*)cm; *shift = shx; *shift_y = shy; *w = cw; *words = nw;
      return GM_OK;
    };
    rc = bitmap(CM_WORDS_MAX, &ix->dev.cm, &ix->dev.cm_shift, &ix->dev.cm_shift_y, &ix->dev.cm_w, &ix->dev.cm_words);
    if (!rc) rc = bitmap(RM_WORDS_MAX, &ix->dev.rm, &ix->dev.rm_shift, &ix->dev.rm_shift_y, &ix->dev.rm_w, &ix->dev.rm_words);
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
  const int64_t cells_per_poly = cells_per_poly_in > 0 ? cells_per_poly_in : 16384;
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
      rc = make_shortcut(ix);   // first: it sets the reference bounds entry_poly checks
      if (!rc) rc = make_list_poly(ix);
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
  rc = make_shortcut(ix);   // first: it sets the reference bounds entry_poly checks
  if (!rc) rc = make_list_poly(ix);
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
  int rc = make_shortcut(ix);   // first: it sets the reference bounds entry_poly checks
  if (!rc) rc = make_list_poly(ix);
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


}  // extern "C"
