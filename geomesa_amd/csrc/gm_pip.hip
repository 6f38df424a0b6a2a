// gm_pip.hip -- st_contains(polygon, point) join on gfx950 with JTS 1.20 semantics.
//
// Reference path: ST_Contains = geom1.contains(geom2) (geomesa-spark-jts/.../udf/SpatialRelationFunctions.scala:29)
// evaluated per candidate pair by GeoMesaJoinRelation.sweeplineJoin / OverlapAction
// (geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91, OverlapAction.scala:25-41) after grid
// partitioning (RelationUtils.scala:30-157).  JTS Geometry.contains(point): envelope covers, then
// relate -> PointLocator with the Mod-2 boundary rule; rings via RayCrossingCounter with the robust
// CGAlgorithmsDD orientation (filter + double-double).  Boundary points are NOT contained.
//
// Index (built once on the host from the polygon CSR, uploaded; the analogue of broadcasting the
// polygon side):
//   * uniform grid over the polygon set's envelope; every (cell, polygon) whose envelopes meet is
//     classified INTERIOR (no edge of the polygon touches the closed cell, cell inside: every point
//     of the cell is contained -- no edge test at all), EXTERIOR (dropped) or BOUNDARY (exact test);
//   * per ring: y-slab buckets of its segments, so a BOUNDARY test only visits the segments whose
//     y-range holds the point's y -- the only ones RayCrossingCounter.countSegment can count.
// The classification is exact: a closed cell that no segment bbox meets lies in one connected
// component of the plane minus the polygon boundary, and every segment straddling a point's y in
// such a cell is at least a cell away, where the JTS orientation filter is already exact.
#include <math.h>
#include <string.h>

#include <algorithm>
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
  const double* poly_env;       // 4 per polygon (minx, miny, maxx, maxy)
  const int32_t* poly_part_off;
  const int32_t* part_ring_off;
  const RingDev* rings;
  const int32_t* slab_off;
  const Edge* edges;
  const int32_t* cell_off;
  const int32_t* cell_ent;      // poly | kind << 30 (kind 1 = interior, 2 = boundary)
  double gx0, gy0, gx1, gy1, inv_cw, inv_ch;
  int32_t gx, gy;
};

__device__ __forceinline__ int cell_of(double v, double v0, double inv, int g) {
  const double c = floor(__dmul_rn(__dsub_rn(v, v0), inv));
  if (!(c >= 0.0)) return 0;
  if (c >= (double)g) return g - 1;
  return (int)c;
}

// RayCrossingCounter.locatePointInRing over the point's slab (PointLocator.locateInPolygonRing
// first rejects points outside the ring envelope)
__device__ int locate_ring(const PipDev& d, int r, double px, double py) {
  const RingDev rd = d.rings[r];
  if (!(px >= rd.minx && px <= rd.maxx && py >= rd.miny && py <= rd.maxy)) return LOC_EXTERIOR;
  const int s = cell_of(py, rd.y0, rd.inv_h, rd.ns);
  const int e0 = d.slab_off[rd.slab_base + s], e1 = d.slab_off[rd.slab_base + s + 1];
  int crossings = 0;
  for (int e = e0; e < e1; ++e) {
    const Edge g = d.edges[e];
    if (g.p1x < px && g.p2x < px) continue;
    if (px == g.p2x && py == g.p2y) return LOC_BOUNDARY;
    if (g.p1y == py && g.p2y == py) {
      double mn = g.p1x, mx = g.p2x;
      if (mn > mx) { mn = g.p2x; mx = g.p1x; }
      if (px >= mn && px <= mx) return LOC_BOUNDARY;
      continue;
    }
    if (((g.p1y > py) && (g.p2y <= py)) || ((g.p2y > py) && (g.p1y <= py))) {
      int orient = jts_orientation(g.p1x, g.p1y, g.p2x, g.p2y, px, py);
      if (orient == 0) return LOC_BOUNDARY;
      if (g.p2y < g.p1y) orient = -orient;
      if (orient == 1) crossings++;
    }
  }
  return (crossings & 1) ? LOC_INTERIOR : LOC_EXTERIOR;
}

// PointLocator.locate over the polygon's components (Mod-2 rule) with locateInPolygon per part
__device__ int locate_poly(const PipDev& d, int poly, double px, double py) {
  const int p0 = d.poly_part_off[poly], p1 = d.poly_part_off[poly + 1];
  bool is_in = false;
  int nb = 0;
  for (int p = p0; p < p1; ++p) {
    const int r0 = d.part_ring_off[p], r1 = d.part_ring_off[p + 1];
    if (r1 <= r0) continue;
    int loc = locate_ring(d, r0, px, py);
    if (loc == LOC_INTERIOR) {
      for (int r = r0 + 1; r < r1; ++r) {
        const int hl = locate_ring(d, r, px, py);
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

// Geometry.contains(point) for candidate entry e of the point's cell
__device__ __forceinline__ bool entry_contains(const PipDev& d, int32_t e, double px, double py) {
  const int poly = e & 0x3fffffff;
  if ((e >> 30) == 1) return true;
  const double* env = d.poly_env + 4 * (int64_t)poly;
  if (!(px >= env[0] && px <= env[2] && py >= env[1] && py <= env[3])) return false;
  return locate_poly(d, poly, px, py) == LOC_INTERIOR;
}

constexpr int JTPB = 512;
constexpr int JCAP = 8192;  // LDS pair staging per block (8 B each: 64 KiB -> 2 blocks per CU)

// one point per lane per tile; persistent grid-stride over tiles of JTPB points
template <bool WRITE>
__global__ __launch_bounds__(JTPB) void k_pip_join(const double* __restrict__ px, const double* __restrict__ py,
                                                   int64_t n, int64_t id_base, PipDev d, int64_t* __restrict__ pt_ids,
                                                   int32_t* __restrict__ poly_ids, int64_t cap,
                                                   unsigned long long* __restrict__ counter) {
  __shared__ uint32_t s_pt[WRITE ? JCAP : 1];
  __shared__ int32_t s_poly[WRITE ? JCAP : 1];
  __shared__ int s_n;
  __shared__ unsigned long long s_base;
  __shared__ int s_cnt;
  if (threadIdx.x == 0) { s_n = 0; s_cnt = 0; }
  __syncthreads();
  const int64_t ntiles = (n + JTPB - 1) / JTPB;
  int my_count = 0;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t i = tile * JTPB + threadIdx.x;
    if (i < n) {
      const double x = __builtin_nontemporal_load(&px[i]);
      const double y = __builtin_nontemporal_load(&py[i]);
      if (x >= d.gx0 && x <= d.gx1 && y >= d.gy0 && y <= d.gy1) {
        const int cx = cell_of(x, d.gx0, d.inv_cw, d.gx), cy = cell_of(y, d.gy0, d.inv_ch, d.gy);
        const int64_t c = (int64_t)cy * d.gx + cx;
        const int k0 = d.cell_off[c], k1 = d.cell_off[c + 1];
        for (int k = k0; k < k1; ++k) {
          const int32_t e = d.cell_ent[k];
          if (!entry_contains(d, e, x, y)) continue;
          if (!WRITE) { my_count++; continue; }
          const int off = atomicAdd(&s_n, 1);
          if (off < JCAP) {
            s_pt[off] = (uint32_t)i;
            s_poly[off] = e & 0x3fffffff;
          } else {  // LDS full inside one tile (heavily overlapping polygons): direct write
            const unsigned long long slot = atomicAdd(counter, 1ull);
            if ((int64_t)slot < cap) { pt_ids[slot] = id_base + i; poly_ids[slot] = e & 0x3fffffff; }
          }
        }
      }
    }
    if (WRITE) {
      __syncthreads();
      const int cnt = s_n < JCAP ? s_n : JCAP;
      if (cnt > JCAP / 2 || (tile + gridDim.x >= ntiles && cnt > 0)) {
        if (threadIdx.x == 0) s_base = atomicAdd(counter, (unsigned long long)cnt);
        __syncthreads();
        for (int j = threadIdx.x; j < cnt; j += JTPB) {
          const int64_t slot = (int64_t)s_base + j;
          if (slot < cap) { pt_ids[slot] = id_base + (int64_t)s_pt[j]; poly_ids[slot] = s_poly[j]; }
        }
        __syncthreads();
        if (threadIdx.x == 0) s_n = 0;
      }
      __syncthreads();
    }
  }
  if (!WRITE) {
    // wave reduce then one LDS add per wave, one global add per block
    for (int off = 32; off > 0; off >>= 1) my_count += __shfl_down(my_count, off, 64);
    if ((threadIdx.x & 63) == 0 && my_count) atomicAdd(&s_cnt, my_count);
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(counter, (unsigned long long)s_cnt);
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

struct gm_pip_index {
  gm_ctx* ctx = nullptr;
  gm::PipDev dev{};
  std::vector<void*> allocs;
  int32_t n_polys = 0;
  int64_t n_entries = 0, n_edges = 0, n_cells = 0;
};

using namespace gm;

namespace {

template <class T>
int upload(gm_pip_index* ix, const std::vector<T>& v, const T** out) {
  void* p = nullptr;
  GM_HIP(hipMalloc(&p, std::max<size_t>(v.size() * sizeof(T), 16)));
  ix->allocs.push_back(p);
  if (!v.empty()) GM_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  *out = (const T*)p;
  return GM_OK;
}

}  // namespace

extern "C" {

int gm_pip_index_create(gm_ctx* ctx, const gm_polyset* ps, gm_pip_index** out) {
  if (!ctx || !ps || !out || ps->n_polys < 0) return GM_E_INVALID;
  *out = nullptr;
  const int P = ps->n_polys;
  if (P > 0 && (!ps->poly_part_off || !ps->part_ring_off || !ps->ring_vert_off)) return GM_E_INVALID;
  const int n_parts = P ? ps->poly_part_off[P] : 0;
  const int n_rings = n_parts ? ps->part_ring_off[n_parts] : 0;
  const int n_verts = n_rings ? ps->ring_vert_off[n_rings] : 0;
  if (n_verts > 0 && (!ps->vx || !ps->vy)) return GM_E_INVALID;

  // ---- rings: envelopes + y-slab segment buckets
  std::vector<RingDev> rings((size_t)n_rings);
  std::vector<int32_t> slab_off;
  std::vector<Edge> edges;
  for (int r = 0; r < n_rings; ++r) {
    const int v0 = ps->ring_vert_off[r], v1 = ps->ring_vert_off[r + 1];
    RingDev& rd = rings[r];
    rd.minx = rd.miny = INFINITY;
    rd.maxx = rd.maxy = -INFINITY;
    for (int v = v0; v < v1; ++v) {
      rd.minx = std::min(rd.minx, ps->vx[v]); rd.maxx = std::max(rd.maxx, ps->vx[v]);
      rd.miny = std::min(rd.miny, ps->vy[v]); rd.maxy = std::max(rd.maxy, ps->vy[v]);
    }
    const int nseg = std::max(0, v1 - v0 - 1);
    int ns = std::max(1, std::min(4096, nseg / 2));
    const double hgt = rd.maxy - rd.miny;
    if (!(hgt > 0.0) || nseg == 0) ns = 1;
    rd.y0 = nseg ? rd.miny : 0.0;
    rd.inv_h = (ns > 1) ? (double)ns / hgt : 0.0;
    rd.ns = ns;
    rd.slab_base = (int32_t)slab_off.size();
    std::vector<std::vector<int32_t>> buckets((size_t)ns);
    for (int j = 0; j < nseg; ++j) {
      const int i = v0 + 1 + j;
      const double ya = ps->vy[i], yb = ps->vy[i - 1];
      const int s0 = host::cell_of(std::min(ya, yb), rd.y0, rd.inv_h, ns);
      const int s1 = host::cell_of(std::max(ya, yb), rd.y0, rd.inv_h, ns);
      for (int k = s0; k <= s1; ++k) buckets[k].push_back(j);
    }
    // slab-major copies of the segments: a slab's segments are contiguous (32 B each)
    for (int k = 0; k < ns; ++k) {
      slab_off.push_back((int32_t)edges.size());
      for (int32_t j : buckets[k]) {
        const int i = v0 + 1 + j;
        edges.push_back(Edge{ps->vx[i], ps->vy[i], ps->vx[i - 1], ps->vy[i - 1]});
      }
    }
  }
  slab_off.push_back((int32_t)edges.size());

  // ---- polygon envelopes (JTS: Polygon envelope = shell envelope; MultiPolygon = union)
  std::vector<double> env((size_t)P * 4);
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

  // ---- grid
  const double W = any ? G[2] - G[0] : 0.0, H = any ? G[3] - G[1] : 0.0;
  int64_t target = std::min<int64_t>(std::max<int64_t>((int64_t)P * 1024, 64), (int64_t)1 << 24);
  int gx = 1, gy = 1;
  if (W > 0 && H > 0) {
    gx = (int)std::max<double>(1.0, std::floor(std::sqrt((double)target * W / H)));
    gy = (int)std::max<int64_t>(1, target / gx);
  } else if (W > 0) {
    gx = (int)std::min<int64_t>(target, 1 << 20);
  } else if (H > 0) {
    gy = (int)std::min<int64_t>(target, 1 << 20);
  }
  const double inv_cw = W > 0 ? (double)gx / W : 0.0, inv_ch = H > 0 ? (double)gy / H : 0.0;
  const double epsx = W > 0 ? W * 1e-9 : 1e-9, epsy = H > 0 ? H * 1e-9 : 1e-9;
  const int64_t ncell = (int64_t)gx * gy;

  // ---- (cell, polygon) classification
  std::vector<int32_t> counts((size_t)ncell + 1, 0);
  struct Ent { int64_t cell; int32_t e; };
  std::vector<Ent> ents;
  for (int p = 0; p < P && any; ++p) {
    const double* e = &env[4 * (size_t)p];
    if (!(e[0] <= e[2])) continue;
    const int cx0 = host::cell_of(e[0], G[0], inv_cw, gx), cx1 = host::cell_of(e[2], G[0], inv_cw, gx);
    const int cy0 = host::cell_of(e[1], G[1], inv_ch, gy), cy1 = host::cell_of(e[3], G[1], inv_ch, gy);
    const int bw = cx1 - cx0 + 1, bh = cy1 - cy0 + 1;
    std::vector<uint8_t> bnd((size_t)bw * bh, 0);
    for (int q = ps->poly_part_off[p]; q < ps->poly_part_off[p + 1]; ++q)
      for (int r = ps->part_ring_off[q]; r < ps->part_ring_off[q + 1]; ++r)
        for (int v = ps->ring_vert_off[r] + 1; v < ps->ring_vert_off[r + 1]; ++v) {
          const double ax = ps->vx[v - 1], ay = ps->vy[v - 1], bx = ps->vx[v], by = ps->vy[v];
          int a0 = host::cell_of(std::min(ax, bx) - epsx, G[0], inv_cw, gx) - cx0;
          int a1 = host::cell_of(std::max(ax, bx) + epsx, G[0], inv_cw, gx) - cx0;
          int b0 = host::cell_of(std::min(ay, by) - epsy, G[1], inv_ch, gy) - cy0;
          int b1 = host::cell_of(std::max(ay, by) + epsy, G[1], inv_ch, gy) - cy0;
          a0 = std::max(a0, 0); b0 = std::max(b0, 0); a1 = std::min(a1, bw - 1); b1 = std::min(b1, bh - 1);
          for (int yy = b0; yy <= b1; ++yy)
            for (int xx = a0; xx <= a1; ++xx) bnd[(size_t)yy * bw + xx] = 1;
        }
    for (int yy = 0; yy < bh; ++yy) {
      int run_loc = -1;
      for (int xx = 0; xx < bw; ++xx) {
        const int64_t cell = (int64_t)(cy0 + yy) * gx + (cx0 + xx);
        int kind;
        if (bnd[(size_t)yy * bw + xx]) {
          kind = 2;
          run_loc = -1;
        } else {
          if (run_loc < 0) {
            // any point of the cell: its nominal centre, checked to map back to the cell
            const double cxm = G[0] + ((double)(cx0 + xx) + 0.5) / inv_cw;
            const double cym = G[1] + ((double)(cy0 + yy) + 0.5) / inv_ch;
            if ((inv_cw > 0 && host::cell_of(cxm, G[0], inv_cw, gx) != cx0 + xx) ||
                (inv_ch > 0 && host::cell_of(cym, G[1], inv_ch, gy) != cy0 + yy) || inv_cw == 0 || inv_ch == 0) {
              kind = 2;
              ents.push_back(Ent{cell, (int32_t)(p | (kind << 30))});
              counts[cell + 1]++;
              continue;
            }
            run_loc = host::locate_poly(ps, p, cxm, cym);
          }
          if (run_loc == LOC_EXTERIOR) continue;
          kind = run_loc == LOC_INTERIOR ? 1 : 2;
        }
        ents.push_back(Ent{cell, (int32_t)(p | (kind << 30))});
        counts[cell + 1]++;
      }
    }
  }
  for (int64_t c = 0; c < ncell; ++c) counts[c + 1] += counts[c];
  std::vector<int32_t> cell_ent(ents.size());
  {
    std::vector<int32_t> fill(counts.begin(), counts.end() - 1);
    for (const Ent& e : ents) cell_ent[fill[e.cell]++] = e.e;  // polys visited in ascending order
  }

  gm_pip_index* ix = new gm_pip_index();
  ix->ctx = ctx;
  ix->n_polys = P;
  ix->n_entries = (int64_t)cell_ent.size();
  ix->n_edges = (int64_t)edges.size();
  ix->n_cells = ncell;
  std::vector<int32_t> ppo(ps->poly_part_off, ps->poly_part_off + P + 1);
  std::vector<int32_t> pro(ps->part_ring_off, ps->part_ring_off + n_parts + 1);
  if (P == 0) { ppo.assign(1, 0); pro.assign(1, 0); }
  int rc = GM_OK;
  GM_HIP(hipSetDevice(ctx->device));
  if (!rc) rc = upload(ix, env, &ix->dev.poly_env);
  if (!rc) rc = upload(ix, ppo, &ix->dev.poly_part_off);
  if (!rc) rc = upload(ix, pro, &ix->dev.part_ring_off);
  if (!rc) rc = upload(ix, rings, &ix->dev.rings);
  if (!rc) rc = upload(ix, slab_off, &ix->dev.slab_off);
  if (!rc) rc = upload(ix, edges, &ix->dev.edges);
  if (!rc) rc = upload(ix, counts, &ix->dev.cell_off);
  if (!rc) rc = upload(ix, cell_ent, &ix->dev.cell_ent);
  if (rc) { gm_pip_index_destroy(ix); return rc; }
  ix->dev.gx0 = G[0]; ix->dev.gy0 = G[1]; ix->dev.gx1 = G[2]; ix->dev.gy1 = G[3];
  ix->dev.inv_cw = inv_cw; ix->dev.inv_ch = inv_ch;
  ix->dev.gx = gx; ix->dev.gy = gy;
  *out = ix;
  return GM_OK;
}

int gm_pip_index_destroy(gm_pip_index* ix) {
  if (!ix) return GM_OK;
  for (void* p : ix->allocs) (void)hipFree(p);
  delete ix;
  return GM_OK;
}

int gm_pip_join(gm_ctx* ctx, const gm_pip_index* ix, const double* px, const double* py, int64_t n, int64_t id_base,
                int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs) {
  if (!ctx || !ix || n < 0 || cap < 0) return GM_E_INVALID;
  const bool write = pt_ids && poly_ids;
  if ((pt_ids == nullptr) != (poly_ids == nullptr)) return GM_E_INVALID;
  if (n > 0 && (!px || !py)) return GM_E_INVALID;
  unsigned long long* counter = (unsigned long long*)ctx->d_scratch;
  GM_HIP(hipMemsetAsync(counter, 0, 8, ctx->stream));
  const int64_t CHUNK = (int64_t)1 << 31;  // LDS staging keeps 32-bit row offsets
  for (int64_t c0 = 0; c0 < n; c0 += CHUNK) {
    const int64_t m = std::min(CHUNK, n - c0);
    const int64_t ntiles = (m + JTPB - 1) / JTPB;
    const unsigned grid = (unsigned)std::min<int64_t>(ntiles, 256 * 2 * 4);
    if (write)
      hipLaunchKernelGGL((k_pip_join<true>), dim3(grid), dim3(JTPB), 0, ctx->stream, px + c0, py + c0, m, id_base + c0,
                         ix->dev, pt_ids, poly_ids, cap, counter);
    else
      hipLaunchKernelGGL((k_pip_join<false>), dim3(grid), dim3(JTPB), 0, ctx->stream, px + c0, py + c0, m, id_base + c0,
                         ix->dev, pt_ids, poly_ids, cap, counter);
    GM_CHECK_LAUNCH();
  }
  if (n_pairs) {
    GM_HIP(hipMemcpyAsync(ctx->h_pinned, counter, 8, hipMemcpyDeviceToHost, ctx->stream));
    GM_HIP(hipStreamSynchronize(ctx->stream));
    *n_pairs = ctx->h_pinned[0];
    if (write && *n_pairs > cap) return GM_E_CAPACITY;
  }
  return GM_OK;
}

}  // extern "C"
