// gm_pip_join.hip -- the st_contains / st_intersects join of device points against a polygon index
// (gm_pip.hpp): the staged direct pass k_pip_join_q, its slab pair output, and the lookup census.
// Reference: GeoMesaJoinRelation.scala:41-91 (sweeplineJoin / buildScan), OverlapAction.scala:25-41,
// the predicate SpatialRelationFunctions.scala:29 (JTS 1.20 Geometry.contains).
#include <algorithm>

#include "gm_arrow.hpp"
#include "gm_pip.hpp"

namespace gm {

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
  // non-temporal: the pair lines are written once and not read back by the join, so they should not
  // take L2 from the coarse and fine words (9.89-9.93 -> 9.83-9.85 ms, profiles/r4/join_nt_ab.txt)
  if (pos < o.cap) { __builtin_nontemporal_store(id, &o.pt[pos]); __builtin_nontemporal_store(poly, &o.pl[pos]); }
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
// One 1024-thread block per CU (16 waves, 6.75 KiB of queues each: the pending fine words live in
// registers) leaves 51.75 KiB of LDS for the coarse EMPTY bitmap (CM_WORDS_MAX: one bit per coarse
// cell up to 424k coarse cells, else per 2 x 1, 2 x 2, ... block; 2 x 1 on the bench's default grid):
// a point whose coarse block is EMPTY costs no gather at all.  The join is bound by the memory
// pipeline (TD busy 94%, the L1 stalled on its outstanding misses 83% of the kernel, r4 PMC): every
// access holds one of the CU's outstanding-miss slots for its latency, so the cost is the count of
// gathers by kind (the gather model); 42% of the bench's points stop at the
// bitmap.
template <bool WRITE, int SRC, bool VEC>
__global__ __launch_bounds__(QTPB) void k_pip_join_q(const double* __restrict__ px, const double* __restrict__ py,
                                                     int64_t n, int64_t id_base, PipDev d, PairOut po,
                                                     int64_t desc_base, ArrowPts ap) {
  constexpr int NW = QTPB / 64;
  __shared__ double s_fx[NW][FCAP], s_fy[NW][FCAP];
  __shared__ uint32_t s_fid[NW][FCAP];
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

  // Pair staging: the wave's pending pairs sit one per lane in registers, lanes [0, pcnt).  A push moves
  // its hit lanes' pairs, in lane order, into lanes pcnt, pcnt + 1, ... (mod 64) by one backward
  // permute, and every 64 pending pairs leave as ONE coalesced 64-pair write at a 64-aligned position of
  // the wave's slab (ids: four whole 128-B lines, polygons: two).  Storing each push's few hits where they
  // fell -- two partial-line stores per push -- cost the join 2.5 of its 10 ms (a timing build without
  // the stores ran 7.5 ms, profiles/r6/join_pairs_ab.txt).  A full slab takes the next with one atomic.
  uint32_t st_id = 0;
  int st_poly = 0;
  int pcnt = 0;                 // wave-uniform: pending pairs
  auto slab_room = [&]() __attribute__((always_inline)) {   // a slab with room for 64 (fills are multiples of 64)
    if (sfill >= SLAB) {
      unsigned long long b = 0;
      if (lane == 0) b = atomicAdd(po.counter, (unsigned long long)SLAB);
      sbase = (int64_t)__shfl(b, 0, 64);
      sfill = 0;
    }
  };
  auto pair_push = [&](bool hit, uint32_t id, int poly) __attribute__((always_inline)) {
    if (!WRITE) { my_count += hit; return; }
    const uint64_t m = __ballot(hit);
    if (!m) return;
    const int c = __popcll(m);
    const int k = (lane - pcnt) & 63;   // this lane's slot takes the hit of rank k (when k < c)
    const bool take = k < c;
    // a forward permute over all 64 lanes: the hits go to slots pcnt, pcnt + 1, ... in lane order and the
    // other lanes fill the remaining slots, so every slot receives exactly one value
    const int dst = hit ? (pcnt + lanes_below(m)) & 63 : (pcnt + c + lanes_below(~m)) & 63;
    const uint32_t nid = (uint32_t)__builtin_amdgcn_ds_permute(dst << 2, (int)id);
    const int npoly = __builtin_amdgcn_ds_permute(dst << 2, poly);
    if (pcnt + c < 64) {
      if (take) { st_id = nid; st_poly = npoly; }
      pcnt += c;
    } else {
      if (take && lane >= pcnt) { st_id = nid; st_poly = npoly; }   // completes the 64
      slab_room();
      pair_store(po, sbase + sfill + lane, id_base + st_id, st_poly);
      sfill += 64;
      if (take && lane < pcnt) { st_id = nid; st_poly = npoly; }    // the rest wraps to lanes 0, 1, ...
      pcnt += c - 64;
    }
  };
  auto item_push = [&](bool valid, bool is_line, double x, double y, uint32_t id, uint32_t ref) __attribute__((always_inline)) {
    const uint64_t ml = __ballot(valid && is_line), mb = __ballot(valid && !is_line);
    if (!(ml | mb)) return;
    if (GM_REF_BAD(qn + qg + 64 > ICAP)) { if (lane == 0) pip_fault(d, PIP_FAULT_QUEUE); return; }   // cannot happen: < 64 here
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

  // pending fine words: a fine round leaves its window [pb, pb + pc) of the fine queue in place, each
  // lane holding its point's 8-B word in registers (pend_w); the window is resolved in one step and
  // only then released.  The list walk reads its point back from the window.
  int pb = 0, pc = 0;
  bool pend = false;                 // wave-uniform: a window awaits resolution
  bool list_on = false;              // wave-uniform: some lane walks a list
  int l_slot = 0, l_lo = 0, l_n = 0, l_j = 0;
  uint2 pend_w = make_uint2(CELL_EMPTY << 30, 0u);

  for (;;) {
    // every other stage idle: the item stage drains what is left (a line round may hand blobs over)
    const bool idle = !list_on && !pend && fn == 0 && step >= nstep;
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
          if (GM_REF_BAD(li >= (uint64_t)d.n_line)) { pip_fault(d, PIP_FAULT_LINE); loc = LOC_EXTERIOR; }
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
    if (pend) {   // ---- resolve the pending window
      const int slot = pb + lane;
      const bool act = lane < pc;
      pend = false;
      uint2 w8 = make_uint2(CELL_EMPTY << 30, 0u);
      uint32_t id = 0;
      double x = 0.0, y = 0.0;
      if (act) { w8 = pend_w; x = fx[slot]; y = fy[slot]; id = fid[slot]; }
      uint32_t w = w8.x;
      bool ihit = false;   // an inline line decided the point
      if (sc8_inline(w8)) {
        const int cx = cell_of(x, d.gx0, d.inv_cw, d.gx), cy = cell_of(y, d.gy0, d.inv_ch, d.gy);
        const int loc = sc8_locate(w8, x, y, d, cx, cy);
        if (loc >= 0) { ihit = join_hit(d.op, loc); w = CELL_EMPTY << 30; }
        else w = d.cell_word[(int64_t)cy * d.gx + cx];   // near the line: the original word's blob decides
      }
      const uint32_t kind = w >> 30, ref = w & 0x3fffffffu;
      pair_push(kind == CELL_INTERIOR || ihit, id, ihit ? sc8_poly(w8) : (int)ref);
      const bool item = kind == CELL_BOUNDARY;
      item_push(item, item && lines_on && (ref & (BLOB_COMPACT | SC_LINE)) == (BLOB_COMPACT | SC_LINE), x, y, id, ref);
      l_j = 0;
      l_n = 0;
      if (kind == CELL_LIST) {
        l_slot = slot;
        l_lo = 4 * (int)(ref >> 4);
        l_n = (int)(w & 15u);
        if (GM_REF_BAD((int64_t)l_lo + 4 > d.n_list)) { pip_fault(d, PIP_FAULT_LIST); l_n = 0; }
        else if (l_n == LIST_LONG) { l_n = (int)d.list_ent[l_lo]; l_lo += 1; }
        if (GM_REF_BAD(l_n < 0 || (int64_t)l_lo + l_n > d.n_list)) { pip_fault(d, PIP_FAULT_LIST); l_n = 0; }
      }
      list_on = __ballot(l_j < l_n) != 0;
      fn = pb;   // the window is released (its list walks run next, before anything can push to the queue)
      continue;
    }
    const bool streaming = step < nstep;
    if (fn >= FBATCH || (!streaming && fn > 0)) {   // ---- fine round: the newest min(fn, 64) points
      wave_lds_sync();
      const int cnt = min(fn, FBATCH);
      const int a = fn - cnt + lane;
      pend_w = make_uint2(CELL_EMPTY << 30, 0u);
      if (lane < cnt)
        pend_w = d.cell_sc8[(int64_t)cell_of(fy[a], d.gy0, d.inv_ch, d.gy) * d.gx + cell_of(fx[a], d.gx0, d.inv_cw, d.gx)];
      pb = fn - cnt;
      pc = cnt;
      pend = true;
      continue;
    }
    if (streaming) {   // ---- stream step: 2 points per lane, their coarse words together
      uint32_t c0 = CELL_EMPTY << 30, c1 = CELL_EMPTY << 30;
      bool g0 = X0 >= d.gx0 && X0 <= d.gx1 && Y0 >= d.gy0 && Y0 <= d.gy1;   // NaN fails
      bool g1 = X1 >= d.gx0 && X1 <= d.gx1 && Y1 >= d.gy0 && Y1 <= d.gy1;
      // every lane computes its cells (clamped, NaN -> 0; unused outside the grid): no branch around them
      const int cx0 = cell_of(X0, d.gx0, d.inv_cw, d.gx), cy0 = cell_of(Y0, d.gy0, d.inv_ch, d.gy);
      const int cx1 = cell_of(X1, d.gx0, d.inv_cw, d.gx), cy1 = cell_of(Y1, d.gy0, d.inv_ch, d.gy);
      if (cm_words) {   // EMPTY coarse blocks from the LDS bitmap: no gather
        const int b0 = ((cy0 >> CF_LOG) >> d.cm_shift_y) * d.cm_w + ((cx0 >> CF_LOG) >> d.cm_shift);
        const int b1 = ((cy1 >> CF_LOG) >> d.cm_shift_y) * d.cm_w + ((cx1 >> CF_LOG) >> d.cm_shift);
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
      if (GM_REF_BAD(fn + 128 > FCAP)) { if (lane == 0 && (m0 | m1)) pip_fault(d, PIP_FAULT_QUEUE); }   // cannot happen: fn < 128
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
    if (pcnt > 0) {   // the last pending pairs: a partial slab (k_pair_plan closes the hole behind them)
      slab_room();
      if (lane < pcnt) pair_store(po, sbase + sfill + lane, id_base + st_id, st_poly);
      sfill += pcnt;
    }
    if (lane == 0) po.desc[desc_base + (int64_t)blockIdx.x * NW + wv] = make_longlong2(sbase, sfill);
  } else {
    for (int off = 32; off > 0; off >>= 1) my_count += __shfl_down(my_count, off, 64);
    if (lane == 0 && my_count) atomicAdd(po.counter, (unsigned long long)my_count);
  }
}

// ------------------------------------------------------------------ lookup census (diagnostic)
// How the join's lookup chain resolves a batch of points, stage by stage (gm_pip_join_census): the
// design numbers behind its gather costs.  Counters (JC_*) are summed per block in LDS.
enum : int {
  JC_POINTS = 0, JC_OUTSIDE, JC_COARSE_EMPTY, JC_COARSE_INTERIOR, JC_COARSE_RAW_MIXED, JC_FINE, JC_FINE_EMPTY,
  JC_FINE_INTERIOR, JC_FINE_LINE, JC_FINE_COMPACT, JC_FINE_GENERIC, JC_FINE_LIST, JC_LIST_ENTRIES,
  JC_LIST_BLOBS, JC_LINE_RESOLVED, JC_LINE_FALLBACK, JC_FINE_INLINE, JC_INLINE_FALLBACK, JC_COARSE_GATHER, JC_FINE_INLINE2, JC_N
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
    // the join's LDS bitmap answers EMPTY coarse blocks without the coarse gather (when it fits)
    bool bm_empty = false;
    if (d.cm_words > 0 && d.cm_words <= CM_WORDS_MAX) {
      const int b = ((cy >> CF_LOG) >> d.cm_shift_y) * d.cm_w + ((cx >> CF_LOG) >> d.cm_shift);
      bm_empty = (d.cm[b >> 5] >> (b & 31)) & 1u;
    }
    if (!bm_empty) c[JC_COARSE_GATHER]++;
    const uint32_t raw = d.coarse_sc[(int64_t)(cy >> CF_LOG) * d.gxc + (cx >> CF_LOG)];
    if ((raw >> 30) == CELL_LIST) c[JC_COARSE_RAW_MIXED]++;
    uint32_t w = coarse_mask(raw, cx, cy, d.coarse_fmt);
    if ((w >> 30) == CELL_EMPTY) { c[JC_COARSE_EMPTY]++; continue; }
    if ((w >> 30) == CELL_INTERIOR) { c[JC_COARSE_INTERIOR]++; continue; }
    c[JC_FINE]++;
    const uint2 w8 = d.cell_sc8[(int64_t)cy * d.gx + cx];
    if (sc8_inline(w8)) {   // one inline line (counted apart from the line entries)
      c[JC_FINE_INLINE]++;
      if ((w8.y >> 30) == 2u) c[JC_FINE_INLINE2]++;
      if (sc8_locate(w8, x, y, d, cx, cy) < 0) c[JC_INLINE_FALLBACK]++;
      continue;
    }
    w = w8.x;
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

// rows per join pass: 2^31 (32-bit row ids in the queues), lowered by the context's
// GM_PARAM_JOIN_CHUNK and kept even, so that every chunk of 16-B aligned columns starts 16-B aligned
static int64_t join_chunk(const gm_ctx* ctx) {
  const int64_t limit = (int64_t)1 << 31;
  const int64_t c = ctx->join_chunk > 0 ? std::min<int64_t>(limit, ctx->join_chunk) : limit;
  return std::max<int64_t>(2, c & ~(int64_t)1);
}

// The staged direct pass over n rows in chunks (join_chunk).  With outputs, each chunk's waves write
// slabs, then k_pair_plan / k_pair_move close the holes, so [0, counter[0]) is contiguous before the
// next chunk reserves past it.  SRC / VEC as k_pip_join_q; `ap` is the Arrow column (tuple bytes `tb`)
// when SRC != 0.
template <int SRC, bool VEC>
static int join_staged(gm_ctx* ctx, const double* px, const double* py, ArrowPts ap, size_t tb, int64_t n,
                       int64_t id_base, const PipDev& dv, int64_t* pt_ids, int32_t* poly_ids, int64_t cap,
                       unsigned long long* counter) {
  const bool write = pt_ids && poly_ids;
  const int64_t CHUNK = join_chunk(ctx);
  const int resident = write ? resident_blocks((const void*)k_pip_join_q<true, SRC, VEC>, ctx->device, QTPB, 1)
                             : resident_blocks((const void*)k_pip_join_q<false, SRC, VEC>, ctx->device, QTPB, 1);
  auto grid_of = [&](int64_t m) {
    const int64_t wsteps = ((m + 1) / 2 + 63) / 64;   // 128-point stream steps, one wave each
    const int64_t blocks = (wsteps + QTPB / 64 - 1) / (QTPB / 64);
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(resident, blocks));
  };
  // the most waves any chunk launches (the first chunk is the largest)
  const int64_t wmax = (int64_t)grid_of(std::min(CHUNK, n)) * (QTPB / 64);
  if (write && wmax > PLAN_MAX) return hip_fail(hipErrorInvalidValue, "join: more waves than the pair plan holds");
  PairOut po{pt_ids, poly_ids, cap, nullptr, nullptr, 0, counter, nullptr};
  PairPlan* plan = nullptr;
  if (write) {   // context workspace: overflow ids | overflow polygons | wave descriptors | plan
    // reservations run at most one partial slab per launched wave past the pair count, so positions
    // in [cap, cap + wmax * SLAB) hold every pair below n_pairs when n_pairs <= cap
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
    const unsigned grid = grid_of(m);
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

// the pair count and the device reference checks of a finished join (synchronises the stream); without
// n_pairs the call stays stream-ordered and a fault waits in the context's sticky word
static int join_result(gm_ctx* ctx, const char* what, unsigned long long* counter, bool write, int64_t cap,
                       int64_t* n_pairs) {
  if (!n_pairs) return GM_OK;
  GM_HIP(hipMemcpyAsync(ctx->h_pinned, counter, 8, hipMemcpyDeviceToHost, ctx->stream));
  const int rc = take_fault(ctx, what);   // synchronises
  if (rc) return rc;
  const int64_t total = ctx->h_pinned[0];
  *n_pairs = total;
  return (write && total > cap) ? GM_E_CAPACITY : GM_OK;
}

static bool join_mode_ok(int mode) {
  if (mode == GM_JOIN_AUTO || mode == GM_JOIN_DIRECT) return true;
  set_error("gm_pip_join: unknown join strategy (GM_JOIN_AUTO or GM_JOIN_DIRECT)");
  return false;
}

}  // namespace gm

using namespace gm;

extern "C" {

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
  if (!join_mode_ok(mode)) return GM_E_INVALID;
  const bool write = pt_ids && poly_ids;
  if ((pt_ids == nullptr) != (poly_ids == nullptr)) return GM_E_INVALID;
  if (n > 0 && (!px || !py)) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  PipDev dv = ix->dev;
  dv.op = predicate == GM_SPATIAL_INTERSECTS ? JOIN_INTERSECTS : JOIN_CONTAINS;
  unsigned long long* counter = (unsigned long long*)ctx->d_scratch;
  dv.fault = (uint32_t*)(ctx->d_scratch + SCRATCH_FAULT);   // sticky reference-check bits (PIP_FAULT_*)
  note_fault_call(ctx, FC_JOIN);
  GM_HIP(hipMemsetAsync(counter, 0, 8, ctx->stream));
  if (n > 0) {
    // chunks start at even rows, so 16-B aligned columns stay aligned in every chunk
    const int rc = aligned16(px) && aligned16(py)
                       ? join_staged<0, true>(ctx, px, py, ArrowPts{}, 16, n, id_base, dv, pt_ids, poly_ids, cap, counter)
                       : join_staged<0, false>(ctx, px, py, ArrowPts{}, 16, n, id_base, dv, pt_ids, poly_ids, cap, counter);
    if (rc) return rc;
  }
  return join_result(ctx, "gm_pip_join", counter, write, cap, n_pairs);
}

int gm_pip_join_arrow(gm_ctx* ctx, const gm_pip_index* ix, const gm_geom_column* pts, int64_t n, int64_t id_base,
                      int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode, int predicate) {
  if (!ctx || !ix || n < 0 || cap < 0 || !pts) return GM_E_INVALID;
  if (predicate != GM_SPATIAL_CONTAINS && predicate != GM_SPATIAL_INTERSECTS) return GM_E_INVALID;
  if (pts->type != GM_GEOM_POINT || (pts->ordinal_bits != 64 && pts->ordinal_bits != 32)) return GM_E_INVALID;
  if (n > 0 && !pts->coords) return GM_E_INVALID;
  if ((pt_ids == nullptr) != (poly_ids == nullptr)) return GM_E_INVALID;
  if (!join_mode_ok(mode)) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  const ArrowPts ap{pts->coords, pts->validity, pts->validity_offset, pts->flip_axis, pts->ordinal_bits == 32};
  PipDev dv = ix->dev;
  dv.op = predicate == GM_SPATIAL_INTERSECTS ? JOIN_INTERSECTS : JOIN_CONTAINS;
  unsigned long long* counter = (unsigned long long*)ctx->d_scratch;
  dv.fault = (uint32_t*)(ctx->d_scratch + SCRATCH_FAULT);
  note_fault_call(ctx, FC_JOIN_ARROW);
  GM_HIP(hipMemsetAsync(counter, 0, 8, ctx->stream));
  if (n > 0) {   // the tuples are read in place (16 B per Float8 tuple, 8 B per Float4 tuple)
    const int rc = ap.f32 ? join_staged<2, false>(ctx, nullptr, nullptr, ap, 8, n, id_base, dv, pt_ids, poly_ids, cap, counter)
                          : join_staged<1, false>(ctx, nullptr, nullptr, ap, 16, n, id_base, dv, pt_ids, poly_ids, cap, counter);
    if (rc) return rc;
  }
  return join_result(ctx, "gm_pip_join_arrow", counter, pt_ids != nullptr, cap, n_pairs);
}

int gm_pip_join_census(gm_ctx* ctx, const gm_pip_index* ix, const double* px, const double* py, int64_t n,
                       int64_t* counters) {
  if (!ctx || !ix || n < 0 || !counters || (n > 0 && (!px || !py))) return GM_E_INVALID;
  GM_HIP(hipSetDevice(ctx->device));
  unsigned long long* d = (unsigned long long*)ctx->d_scratch;
  static_assert(JC_N < SCRATCH_FAULT, "census counters reach the context's fault word");
  GM_HIP(hipMemsetAsync(d, 0, JC_N * 8, ctx->stream));
  if (n > 0) {
    hipLaunchKernelGGL(k_pip_census, dim3((unsigned)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0, ctx->stream,
                       px, py, n, ix->dev, d);
    GM_CHECK_LAUNCH();
  }
  return copy_d2h(ctx, counters, d, JC_N * 8);
}

}  // extern "C"
