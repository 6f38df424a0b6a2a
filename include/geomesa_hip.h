/*
 * geomesa_hip.h -- C ABI of the MI355X-native GeoMesa hot path (libgeomesa_hip.so, gfx950).
 *
 * Drop-in boundary for the Scala/JVM surface of liyq0307/geomesa's spatio-temporal
 * index-and-filter path.  Every entry point names the reference interface it replaces
 * (paths abbreviated: z3/ = geomesa-z3/src/main/scala/org/locationtech/geomesa/,
 *  idx/ = geomesa-index-api/src/main/scala/org/locationtech/geomesa/index/).
 * A JVM binding (JNI or Java FFM) is sketched in INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Array arguments are DEVICE pointers (hipMalloc'd, or
 *    any device allocation of the caller) unless the parameter says "host".  Buffers are
 *    caller-owned; the library never retains a pointer past the call (or past gm_ctx_sync()
 *    for the asynchronous entry points).
 *  - Every call returns an int status: GM_OK (0) or a negative GM_E_* code.
 *  - Per-element failures mirror the JVM exceptions: an optional device uint8 status[] gets
 *    GM_ST_* per element, and an optional host gm_batch_status receives the error count and
 *    the first failing element, so a shim can throw the same IllegalArgumentException the
 *    Scala code throws on the first bad element.  Passing summary = NULL keeps the call
 *    fully asynchronous on the context's stream.
 *  - Thread safety: one gm_ctx per thread; calls on different contexts are independent.
 *  - Configuration knobs the Scala code reads from system properties
 *    (geomesa.scan.ranges.target, geomesa.scan.ranges.recurse, XZ precision g, ...) are
 *    explicit parameters here, never globals.
 */
#ifndef GEOMESA_HIP_H
#define GEOMESA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM_ABI_VERSION 1

/* return codes */
#define GM_OK 0
#define GM_E_INVALID (-1)     /* bad argument (null pointer, bad period/precision, malformed filter) */
#define GM_E_HIP (-2)         /* HIP runtime failure; see gm_last_error() */
#define GM_E_CAPACITY (-3)    /* output capacity too small; the needed size is reported */
#define GM_E_ELEMENT (-4)     /* at least one element failed (only when no status[] and no summary) */
#define GM_E_INDEX (-5)       /* a device-side reference check of a join failed (corrupt or mismatched index,
                                 or a broken internal invariant); the call's output is not valid */

/* per-element status codes */
/* BinnedTime periods (TimePeriod, z3/curve/BinnedTime.scala:283-291) */
#define GM_PERIOD_DAY 0
#define GM_PERIOD_WEEK 1
#define GM_PERIOD_MONTH 2
#define GM_PERIOD_YEAR 3

#define GM_ST_OK 0
#define GM_ST_OUT_OF_BOUNDS 1 /* Z3SFC/Z2SFC/XZ2SFC/XZ3SFC require(...) -> IllegalArgumentException */
#define GM_ST_BAD_TIME 2      /* BinnedTime require(...): before 1970-01-01 or past the period's max date */
#define GM_ST_UNORDERED 3     /* XZ require(xmin <= xmax ...) / ZRange require(min <= max) */
#define GM_ST_NULL_GEOM 4     /* toIndexKey: "Null geometry in feature" (Z3IndexKeySpace.scala:66-68) */

/* TimePeriod (z3/curve/BinnedTime.scala:283-291) */
#define GM_DAY 0
#define GM_WEEK 1
#define GM_MONTH 2
#define GM_YEAR 3

typedef struct gm_ctx gm_ctx;

typedef struct {
  int64_t n_errors;     /* number of failed elements */
  int64_t first_index;  /* index of the first failed element, -1 if none */
  int32_t first_code;   /* GM_ST_* of that element */
  int32_t reserved;
} gm_batch_status;

/* IndexRange (z3/zorder/sfcurve/package.scala:45-76): CoveredRange when contained = 1 */
typedef struct {
  int64_t lower;
  int64_t upper;
  int32_t contained;
  int32_t reserved;
} gm_range;

/* ------------------------------------------------------------------ context */
int gm_abi_version(void);
/* stream: the hipStream_t every call of this context launches on (NULL = the default null stream,
   which is also PyTorch's default stream) */
int gm_ctx_create(int device, void* stream, gm_ctx** out);
/* same, on a new non-blocking stream owned (and destroyed) by the context */
int gm_ctx_create_owned(int device, gm_ctx** out);
int gm_ctx_destroy(gm_ctx* ctx);
/* waits for the context stream; GM_E_INDEX when a stream-ordered polygon-index call since the last
   check failed its device reference checks (gm_pip_join without n_pairs, gm_pip_relate) */
int gm_ctx_sync(gm_ctx* ctx);
void* gm_ctx_stream(gm_ctx* ctx);
const char* gm_last_error(void);
/* per-context tuning parameters (library defaults when unset) */
#define GM_PARAM_JOIN_CHUNK 1   /* points per pass of the join (0 = default 2^31; odd values are rounded
                                   down to even, at least 2); smaller values only add passes -- the
                                   pair set never changes */
#define GM_PARAM_INDEX_BUILD 2  /* where gm_pip_index_create builds the join index: 0 (default) = on the
                                   device (same arrays, byte for byte), 1 = on the host */
#define GM_PARAM_RANGES_CHUNK 3 /* queries per chunk of a batched ranges call whose output is pinned host
                                   memory: chunk k's result copy runs while chunk k + 1 computes (0 =
                                   default: one batch below 16384 queries, else about nq / 8 per chunk);
                                   the output never changes */
#define GM_PARAM_SORT_MODE 4    /* gm_sort_keys: 0 (default) = one to four digit passes over the top
                                   ~log2(n) - 1 varying key bits, then every run of equal prefixes ranked
                                   in LDS (digit passes over every varying byte when a run exceeds 256
                                   rows); 1 = digit passes over every varying byte.  The output never
                                   changes */
#define GM_PARAM_SORT_LAST 5    /* read-only (gm_ctx_get_param): how the context's last gm_sort_keys ran:
                                   digit passes, plus 256 when the runs were ranked locally */
#define GM_PARAM_INDEX_COARSE 6 /* the join's coarse-cell sub-block masks, chosen when a polygon index is
                                   built or imported on this context: -1 (default) = automatic (with
                                   fewer than 2^14 polygons 8 sub-blocks with EMPTY and INTERIOR-of-one-
                                   polygon bits, else 16 EMPTY bits), 0 = EMPTY bits, 1 = EMPTY and
                                   INTERIOR bits.  Results never change */
#define GM_PARAM_INDEX_CORE_RETIRED 7 /* ABI change (round 5): gm_pip_index_core and its parameter 7
                                   (the row predicate's per-polygon core rectangles) were removed with the
                                   rectangles.  Kept for one release as an accepted no-op: setting it
                                   succeeds and changes nothing, reading it returns 0 */
#define GM_PARAM_HIST_GRID 8    /* gm_z3_histogram: workgroups of the LDS-counter kernel (0 = default: one
                                   resident wave of workgroups); fewer workgroups each count more features
                                   and drain their packed counters more often.  Results never change */
#define GM_PARAM_RELATE_ROWS64 9 /* gm_pip_relate: 1 = always the kernel with 64-bit queue rows and the
                                   join's coarse bitmap (the one calls of 2^32 rows or more take);
                                   0 (default) = 32-bit queue rows and the finer bitmap below 2^32 rows.
                                   Results never change */
int gm_ctx_set_param(gm_ctx* ctx, int param, int64_t value);
int gm_ctx_get_param(gm_ctx* ctx, int param, int64_t* value);
/* device memory helpers for callers without their own allocator (e.g. a JNI shim) */
int gm_device_alloc(gm_ctx* ctx, size_t bytes, void** ptr);
int gm_device_free(gm_ctx* ctx, void* ptr);
int gm_copy_to_device(gm_ctx* ctx, void* dst, const void* host_src, size_t bytes);
int gm_copy_to_host(gm_ctx* ctx, void* host_dst, const void* src, size_t bytes);
/* device-to-device copy on the context stream (asynchronous): 16 B per lane with non-temporal loads and
   stores when both pointers are 16-B aligned -- the streaming copy the benchmark calibrates HBM against */
int gm_device_copy(gm_ctx* ctx, void* dst, const void* src, size_t bytes);
/* HIP-event timing on the context stream: brackets any sequence of calls */
int gm_timer_start(gm_ctx* ctx);
int gm_timer_stop(gm_ctx* ctx, float* ms);

/* ------------------------------------------------------------------ Z-curve keys */
/* Z3SFC.index(x, y, t, lenient) (z3/curve/Z3SFC.scala:37-52), t = offset within the period
   (BinnedTime units).  precision = bits per dimension, 1..21 (StandardZ3Dimensions, :92-99). */
int gm_z3_index(gm_ctx* ctx, const double* x, const double* y, const int64_t* t, int64_t n, int period,
                int precision, int lenient, int64_t* z, uint8_t* status, gm_batch_status* summary);

/* Z3IndexKeySpace.toIndexKey lines 71-76 (idx/index/z3/Z3IndexKeySpace.scala): epoch millis ->
   BinnedTime.timeToBinnedTime(period) (z3/curve/BinnedTime.scala:73-86) -> Z3SFC(period).index.
   Produces the [bin][z] key columns (the row key is [shard?][bin BE16][z BE64][id], :81-92). */
int gm_z3_index_key(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n,
                    int period, int lenient, int16_t* bin, int64_t* z, uint8_t* status,
                    gm_batch_status* summary);

/* Z3SFC.invert (z3/curve/Z3SFC.scala:54-57) */
int gm_z3_invert(gm_ctx* ctx, const int64_t* z, int64_t n, int period, int precision, double* x, double* y,
                 int64_t* t);

/* Z2SFC.index / invert (z3/curve/Z2SFC.scala:26-45); precision 1..31 (Z2SFC object uses 31) */
int gm_z2_index(gm_ctx* ctx, const double* x, const double* y, int64_t n, int precision, int lenient,
                int64_t* z, uint8_t* status, gm_batch_status* summary);
int gm_z2_invert(gm_ctx* ctx, const int64_t* z, int64_t n, int precision, double* x, double* y);

/* BinnedTime.timeToBinnedTime(period) (z3/curve/BinnedTime.scala:73-86) */
int gm_binned_time(gm_ctx* ctx, const int64_t* t_ms, int64_t n, int period, int16_t* bin, int64_t* offset,
                   uint8_t* status, gm_batch_status* summary);

/* XZ2SFC(g).index(xmin, ymin, xmax, ymax, lenient) (z3/curve/XZ2SFC.scala:54-77) */
int gm_xz2_index(gm_ctx* ctx, const double* xmin, const double* ymin, const double* xmax, const double* ymax,
                 int64_t n, int g, int lenient, int64_t* out, uint8_t* status, gm_batch_status* summary);
/* XZ3SFC(g, period).index(xmin, ymin, zmin, xmax, ymax, zmax, lenient) (z3/curve/XZ3SFC.scala:53-76) */
int gm_xz3_index(gm_ctx* ctx, const double* xmin, const double* ymin, const double* zmin, const double* xmax,
                 const double* ymax, const double* zmax, int64_t n, int g, int period, int lenient,
                 int64_t* out, uint8_t* status, gm_batch_status* summary);
/* XZ3IndexKeySpace.toIndexKey (idx/index/z3/XZ3IndexKeySpace.scala:60-95) over envelope + dtg columns:
   bin = BinnedTime(period)(dtg) (t_ms NULL = every dtg null -> 0; a bad date fails even when lenient),
   xz = XZ3SFC(g, period).index(xmin, ymin, offset, xmax, ymax, offset, lenient); a failed row gets
   bin 0 and xz 0 and its status */
int gm_xz3_index_key(gm_ctx* ctx, const double* xmin, const double* ymin, const double* xmax, const double* ymax,
                     const int64_t* t_ms, int64_t n, int g, int period, int lenient, int16_t* bin, int64_t* xz,
                     uint8_t* status, gm_batch_status* summary);

/* ------------------------------------------------------------------ range decomposition */
/* Batched ZN.zranges (z3/zorder/sfcurve/ZN.scala:110-242) as reached from Z3SFC.ranges
   (z3/curve/Z3SFC.scala:59-67) and Z2SFC.ranges (z3/curve/Z2SFC.scala:47-52).
   Host inputs, one query per entry of query_off: query q owns boxes [box_off[q], box_off[q+1]) of
   xy (host, 4 doubles each) and, for Z3, times [time_off[q], time_off[q+1]) of t (host, 2 int64
   each, offsets within the period).  The z-bounds of a query are the cross product, as in
   Z3SFC.ranges.  max_ranges <= 0 means None; max_recurse < 0 means the default (Z3:
   Int.MaxValue, Z2: ZN.DefaultRecurse = 7).  Output: ranges of query q are
   out[out_off[q] .. out_off[q+1]) (out_off host); capacity in ranges.  `out` is host memory
   (pageable or pinned; pinned output is copied back chunk by chunk, overlapping the next chunk's
   kernels) or device memory (the ranges stay in HBM for a device-side consumer: no copy).  Returns
   GM_E_CAPACITY with *needed set when cap is too small.  The same output rules hold for
   gm_z2_ranges, gm_zranges, gm_xz2_ranges and gm_xz3_ranges. */
int gm_z3_ranges(gm_ctx* ctx, int64_t n_queries, const int32_t* box_off, const double* xy,
                 const int32_t* time_off, const int64_t* t, int period, int precision, int range_precision,
                 int max_ranges, int max_recurse, int64_t* out_off, gm_range* out, int64_t cap,
                 int64_t* needed, int32_t* query_status);
int gm_z2_ranges(gm_ctx* ctx, int64_t n_queries, const int32_t* box_off, const double* xy, int precision,
                 int range_precision, int max_ranges, int max_recurse, int64_t* out_off, gm_range* out,
                 int64_t cap, int64_t* needed, int32_t* query_status);
/* ZN.zranges(zbounds: Array[ZRange], precision, maxRanges, maxRecurse) (z3/zorder/sfcurve/ZN.scala:110-242)
   on raw z bounds, as Z3.zranges (dims = 3) / Z2.zranges (dims = 2), batched: query q owns the bounds
   [bound_off[q], bound_off[q+1]) of zbounds (host, (min, max) int64 pairs).  max_ranges <= 0 = None;
   max_recurse < 0 = the Scala default Some(ZN.DefaultRecurse) = 7 (ZN.scala:113).  A bound with
   min > max gets query status GM_ST_UNORDERED (ZRange's require, z3/zorder/sfcurve/package.scala:24).
   Outputs as gm_z3_ranges. */
int gm_zranges(gm_ctx* ctx, int dims, int64_t n_queries, const int32_t* bound_off, const int64_t* zbounds,
               int range_precision, int max_ranges, int max_recurse, int64_t* out_off, gm_range* out, int64_t cap,
               int64_t* needed, int32_t* query_status);
/* Batched XZ2SFC.ranges / XZ3SFC.ranges (z3/curve/XZ2SFC.scala:130-252, XZ3SFC.scala:139-262);
   windows as above (4 or 6 doubles each, user space). */
int gm_xz2_ranges(gm_ctx* ctx, int64_t n_queries, const int32_t* win_off, const double* windows, int g,
                  int max_ranges, int64_t* out_off, gm_range* out, int64_t cap, int64_t* needed,
                  int32_t* query_status);
int gm_xz3_ranges(gm_ctx* ctx, int64_t n_queries, const int32_t* win_off, const double* windows, int g,
                  int period, int max_ranges, int64_t* out_off, gm_range* out, int64_t cap, int64_t* needed,
                  int32_t* query_status);

/* ------------------------------------------------------------------ filter scans */
/* Z3Filter.inBounds over columnar keys (idx/filters/Z3Filter.scala:26-62), RowFilterIterator's
   per-row call (geomesa-accumulo-iterators/.../RowFilterIterator.scala:57) as one pass.
   filter_bytes (host) is exactly Z3Filter.serializeToBytes (Z3Filter.scala:112-137).
   bin_ranges (host, n_bin_ranges pairs of int16, inclusive) restricts the scan to the query's
   epochs (the bins Z3IndexKeySpace.getRanges scans, Z3IndexKeySpace.scala:161-194);
   n_bin_ranges = 0 scans every bin.
   Outputs (device, each optional): mask = 1 bit per row (bit i%64 of word i/64, ceil(n/64) words),
   ids = compacted matching row indices (ids_cap entries, in ascending order).
   *n_match (host) receives the match count (this call synchronises when n_match != NULL). */
int gm_z3filter_scan(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const int16_t* bin_ranges,
                     int n_bin_ranges, const int16_t* bin, const int64_t* z, int64_t n, uint64_t* mask,
                     int64_t* ids, int64_t ids_cap, int64_t* n_match);
/* Z2Filter.inBounds (idx/filters/Z2Filter.scala:20-35) */
int gm_z2filter_scan(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const int64_t* z, int64_t n,
                     uint64_t* mask, int64_t* ids, int64_t ids_cap, int64_t* n_match);
/* RowFilter.inBounds(buf, offset) on row-key BYTES (idx/filters/RowFilter.scala:11-13), the loop of
   RowFilterIterator.findTop (geomesa-accumulo-iterators/.../RowFilterIterator.scala:52-66) and
   Z3HBaseFilter as one pass: row i is rows[row_off[i] .. row_off[i+1]) (device bytes; device int64
   offsets, n + 1 of them) and its key starts at key_offset (RowFilterIterator.RowOffsetKey, the
   shard / table-sharing prefix length).  Z3Filter.inBounds (Z3Filter.scala:26-28) reads the
   big-endian short epoch at key_offset and the long z at key_offset + 2; Z2Filter.inBounds
   (Z2Filter.scala:22-35) the long at key_offset.  A row shorter than its key never matches and is
   counted in *n_short (host, optional; the JVM read throws ArrayIndexOutOfBoundsException).
   Outputs as gm_z3filter_scan (no bin restriction: the scan ranges already chose the rows). */
int gm_z3filter_scan_rows(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const uint8_t* rows,
                          const int64_t* row_off, int key_offset, int64_t n, uint64_t* mask, int64_t* ids,
                          int64_t ids_cap, int64_t* n_match, int64_t* n_short);
int gm_z2filter_scan_rows(gm_ctx* ctx, const uint8_t* filter_bytes, size_t filter_len, const uint8_t* rows,
                          const int64_t* row_off, int key_offset, int64_t n, uint64_t* mask, int64_t* ids,
                          int64_t ids_cap, int64_t* n_match, int64_t* n_short);
/* Strict full-filter evaluation on raw columns (useFullFilter, Z3IndexKeySpace.scala:240-254):
   GeoTools BBOX on a point (geomesa-filter/.../GeometryProcessing.scala:129, inclusive) AND
   FastDuring (geomesa-filter/.../FastTemporalOperator.scala:123-126, exclusive at both ends, ms).
   bbox (host) = xmin, ymin, xmax, ymax; has_during = 0 skips the time test. */
int gm_strict_scan(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n,
                   const double* bbox, int has_during, int64_t during_lo_ms, int64_t during_hi_ms,
                   uint64_t* mask, int64_t* ids, int64_t ids_cap, int64_t* n_match);

/* ------------------------------------------------------------------ st_contains join */
/* Polygon set in CSR form (host arrays): polygon -> parts (a MultiPolygon's components; a
   Polygon has one) -> rings (first ring of each part is the shell, the rest are holes) ->
   vertices.  Rings are closed (first vertex == last vertex), as JTS LinearRings are. */
typedef struct {
  int32_t n_polys;
  const int32_t* poly_part_off; /* [n_polys + 1] */
  const int32_t* part_ring_off; /* [n_parts + 1] */
  const int32_t* ring_vert_off; /* [n_rings + 1] */
  const double* vx;             /* [n_verts] */
  const double* vy;             /* [n_verts] */
} gm_polyset;

typedef struct gm_pip_index gm_pip_index;

/* Uploads the polygon set and builds the device-side join index (uniform grid over polygon
   envelopes -- the analogue of RelationUtils.grid, geomesa-spark-sql/.../RelationUtils.scala:30-157 --
   plus per-ring y-slab edge buckets). */
int gm_pip_index_create(gm_ctx* ctx, const gm_polyset* polys, gm_pip_index** out);
/* same with an explicit grid density: ~cells_per_poly grid cells per polygon over the set's
   envelope (0 = default 16384, at most 2^26 cells; a coarse 8x8-cell table in front of it stays
   L2-resident) */
int gm_pip_index_create_ex(gm_ctx* ctx, const gm_polyset* polys, int cells_per_poly, gm_pip_index** out);
int gm_pip_index_destroy(gm_pip_index* index);
/* index statistics: stats[0..6] = cells, (cell, polygon) entries, boundary entries, ring records,
   ring records that fall back to the slab walk, boundary blob bytes, compact (one-line) blobs */
int gm_pip_index_stats(const gm_pip_index* index, int64_t* stats);
/* Diagnostic (no reference counterpart): how the join's lookup chain resolves the device points
   px / py, stage by stage -- counters[20] = points, outside the grid, coarse EMPTY, coarse INTERIOR,
   points in mixed coarse cells before the sub-block masks, fine lookups, fine EMPTY, fine INTERIOR,
   fine line entries, fine compact blobs, fine generic blobs, fine lists, list entries, list entries
   that are blobs, line entries that decide, line entries that fall back to the blob, fine words with
   inline lines, inline words that fall back to the blob, coarse-table gathers (points the LDS
   EMPTY bitmap does not answer), fine words with two inline lines. */
int gm_pip_join_census(gm_ctx* ctx, const gm_pip_index* index, const double* px, const double* py, int64_t n,
                       int64_t* counters);

/* A built index as device arrays, for shipping it to the other GPUs of a join (RCCL broadcast) instead
   of rebuilding it on every rank -- the broadcast side of GeoMesaJoinRelation's join
   (geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91).  gm_pip_index_export fills the layout
   (array sizes + grid scalars, plain host data); gm_pip_index_copy_array copies device array k into a
   caller buffer of layout.bytes[k] bytes (stream-ordered); gm_pip_index_import builds an index on
   ctx's device from the layout and device copies of the arrays (the library copies them: the caller
   keeps ownership of `arrays`). */
#define GM_PIP_INDEX_ARRAYS 8
#define GM_PIP_LAYOUT_VERSION 1
typedef struct {
  int32_t version;                       /* GM_PIP_LAYOUT_VERSION */
  int32_t dims[4];                       /* grid columns, rows, coarse columns, polygons */
  int32_t reserved;
  double grid[6];                        /* grid envelope x0 y0 x1 y1, inverse cell width / height */
  int64_t stats[9];                      /* gm_pip_index_stats[0..6], most boundary / all entries of a cell */
  int64_t bytes[GM_PIP_INDEX_ARRAYS];    /* device bytes of each array */
} gm_pip_index_layout;
int gm_pip_index_export(const gm_pip_index* index, gm_pip_index_layout* layout);
int gm_pip_index_copy_array(gm_ctx* ctx, const gm_pip_index* index, int k, void* dst);
int gm_pip_index_import(gm_ctx* ctx, const gm_pip_index_layout* layout, void* const* arrays, gm_pip_index** out);

/* ST_Contains(polygon, point) = JTS Geometry.contains (geomesa-spark-jts/.../udf/
   SpatialRelationFunctions.scala:29), evaluated for every (point, polygon) pair -- the result of
   GeoMesaJoinRelation.sweeplineJoin + OverlapAction (geomesa-spark-sql/.../GeoMesaJoinRelation.scala:41-91,
   OverlapAction.scala:25-41) as one batch.  Points are device columns.  Matching pairs go to
   pt_ids / poly_ids (device, cap entries; point ids are id_base + row); order within the output is
   unspecified (the reference returns an unordered RDD).  *n_pairs (host) receives the pair count;
   when it exceeds cap, GM_E_CAPACITY is returned and no pair beyond cap is written.  With
   pt_ids = poly_ids = NULL the call only counts.  With n_pairs = NULL the call is stream-ordered
   (asynchronous); with n_pairs it synchronises the context stream.  A device reference check of the
   index that fails (a corrupt or mismatched imported index) makes the output invalid and is reported
   as GM_E_INDEX by the next synchronising call on the context (this join with n_pairs, gm_query_scan,
   gm_ctx_sync). */
int gm_pip_join(gm_ctx* ctx, const gm_pip_index* index, const double* px, const double* py, int64_t n,
                int64_t id_base, int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs);

/* join strategies for gm_pip_join_ex.  Both run the staged direct pass over the point columns; a
   band-partitioned and a two-pass variant measured slower on MI355X and were
   removed, and any other value returns GM_E_INVALID */
#define GM_JOIN_AUTO 0
#define GM_JOIN_DIRECT 1
/* gm_pip_join with an explicit strategy */
int gm_pip_join_ex(gm_ctx* ctx, const gm_pip_index* index, const double* px, const double* py, int64_t n,
                   int64_t id_base, int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode);

/* gm_pip_join_ex with the join's predicate: GM_SPATIAL_CONTAINS (st_contains(polygon, point) /
   st_within(point, polygon): the point in the interior) or GM_SPATIAL_INTERSECTS (st_intersects /
   st_covers: boundary included).  GeoMesaJoinRelation takes any (Geometry, Geometry) => Boolean UDF of
   the join condition (GeoMesaJoinRelation.scala:67-79, SQLRules.scala:186-190); these are the ones with
   a non-empty result over (polygon, point) pairs besides st_touches. */
int gm_pip_join_pred(gm_ctx* ctx, const gm_pip_index* index, const double* px, const double* py, int64_t n,
                     int64_t id_base, int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode,
                     int predicate);

/* ------------------------------------------------------------------ fused query filter */
/* spatial terms of gm_query_scan */
#define GM_SPATIAL_NONE 0
#define GM_SPATIAL_INTERSECTS 1  /* INTERSECTS(geom, P): JTS P.intersects(point), boundary included */
#define GM_SPATIAL_CONTAINS 2    /* CONTAINS(P, geom) / WITHIN(geom, P): JTS P.contains(point), interior only */
/* The full filter of a point query in one pass (useFullFilter, Z3IndexKeySpace.scala:240-254):
   BBOX (inclusive, geomesa-filter/.../GeometryProcessing.scala:129) AND during (exclusive ms,
   FastTemporalOperator.scala:123-126) AND the OR over the polygons of `geoms` of the spatial term
   (GeometryProcessing.process turns a split query geometry into an OR of its parts, :104-136).
   bbox (host xmin, ymin, xmax, ymax) NULL = no BBOX term; has_during = 0 = no time term;
   spatial_op GM_SPATIAL_NONE = no geometry term (geoms may be NULL).  geoms is any polygon index
   (gm_pip_index_create_ex; a denser grid, e.g. 65536 cells for one query polygon, makes more rows
   resolve in one lookup).  Outputs as gm_strict_scan: mask bits, ids ascending, *n_match. */
int gm_query_scan(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n,
                  const double* bbox, int has_during, int64_t during_lo_ms, int64_t during_hi_ms,
                  const gm_pip_index* geoms, int spatial_op, uint64_t* mask, int64_t* ids, int64_t ids_cap,
                  int64_t* n_match);

/* ------------------------------------------------------------------ row-wise predicates (UDF path) */
/* Spark SQL's st_* relation UDFs evaluated row by row (SpatialRelationFunctions.scala:29-37, null in
   -> null out via nullableUDF, SQLFunctionHelper.scala:27-33): row i relates polygon poly[i] of the
   index with point (px[i], py[i]) and gets PointLocator's location of the point in the polygon.
   For an areal geometry and a point every DE-9IM predicate follows from it:
     st_contains(P, pt) = st_within(pt, P) = INTERIOR;  st_covers / st_intersects = not EXTERIOR;
     st_touches = BOUNDARY;  st_disjoint = EXTERIOR;  st_crosses / st_overlaps / st_equals = false.
   poly[i] < 0 or >= the polygon count marks a null row (GM_LOC_NULL).  Device arrays. */
#define GM_LOC_EXTERIOR 0
#define GM_LOC_BOUNDARY 1
#define GM_LOC_INTERIOR 2
#define GM_LOC_NULL 255
/* Stream-ordered; a failed device reference check is reported as for gm_pip_join (GM_E_INDEX at the
   next synchronising call: the locations are then invalid).  gm_query_scan checks its geometry term
   the same way and reports it itself. */
int gm_pip_relate(gm_ctx* ctx, const gm_pip_index* index, const int32_t* poly, const double* px, const double* py,
                  int64_t n, uint8_t* loc);

/* ------------------------------------------------------------------ Arrow columnar input */
/* GeoMesa's Arrow geometry vectors (geomesa-arrow-jts) as zero-copy device input.  A point column is
   a FixedSizeList(2) of Float8 (PointVector) or Float4 (PointFloatVector) whose tuples hold [y, x]
   by default and [x, y] when the vector's flipAxisOrder is set (AbstractPointVector.java:52-79);
   line, polygon and multi-geometry columns nest List offsets around the same tuples
   (AbstractLineStringVector.java, AbstractPolygonVector.java:56-84 -- rings, the first one the
   shell --, AbstractMultiPolygonVector.java:61-95 -- polygons, rings).  Dates are Arrow int64 epoch
   milliseconds.  Null slots come from the Arrow validity bitmaps (LSB bit order). */
#define GM_GEOM_POINT 0
#define GM_GEOM_LINESTRING 1      /* offsets[0]: slot -> tuples */
#define GM_GEOM_POLYGON 2         /* offsets[0]: slot -> rings, offsets[1]: ring -> tuples */
#define GM_GEOM_MULTIPOINT 3      /* offsets[0]: slot -> tuples */
#define GM_GEOM_MULTILINESTRING 4 /* offsets[0]: slot -> lines, offsets[1]: line -> tuples */
#define GM_GEOM_MULTIPOLYGON 5    /* offsets[0]: slot -> polygons, [1]: polygon -> rings, [2]: ring -> tuples */

typedef struct {
  int32_t type;              /* GM_GEOM_* */
  int32_t ordinal_bits;      /* 64 (Float8 vectors) or 32 (Float4 "...FloatVector"s) */
  int32_t flip_axis;         /* 0: [y, x] tuples (the default), 1: [x, y] */
  int32_t reserved;
  const void* coords;        /* tuple ordinates, tuple j at [2j], [2j + 1] (already advanced by the
                                innermost child array's offset) */
  const uint8_t* validity;   /* top-level validity bitmap, NULL = no nulls */
  int64_t validity_offset;   /* bit index of slot 0 in validity (the Arrow array offset) */
  const int32_t* offsets[3]; /* List offsets, outermost first, each advanced by its array's offset;
                                unused levels NULL */
} gm_geom_column;

typedef struct {
  const int64_t* millis;     /* epoch ms (Arrow Timestamp(ms) / Date(ms) / Int64) */
  const uint8_t* validity;   /* NULL = no nulls */
  int64_t validity_offset;
} gm_time_column;

/* Z3IndexKeySpace.toIndexKey over an Arrow batch (idx/index/z3/Z3IndexKeySpace.scala:63-95):
   point column + date column (dtg NULL or a null slot -> time 0, :70).  A null geometry is
   GM_ST_NULL_GEOM (the IllegalArgumentException of :66-68).  Device arrays, as gm_z3_index_key. */
int gm_z3_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, const gm_time_column* dtg, int64_t n,
                          int period, int lenient, int16_t* bin, int64_t* z, uint8_t* status,
                          gm_batch_status* summary);
/* Z2IndexKeySpace.toIndexKey (idx/index/z2/Z2IndexKeySpace.scala:48-75): Z2SFC.index of a point column */
int gm_z2_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, int64_t n, int lenient, int64_t* z,
                          uint8_t* status, gm_batch_status* summary);
/* XZ2IndexKeySpace.toIndexKey (idx/index/z2/XZ2IndexKeySpace.scala:48-76): XZ2SFC(g).index of each
   geometry's JTS envelope (Geometry.getEnvelopeInternal: a polygon's envelope is its shell's, a multi
   geometry's the union of its parts'; an empty geometry has the null envelope -> GM_ST_UNORDERED). */
int gm_xz2_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, int64_t n, int g, int lenient, int64_t* xz,
                           uint8_t* status, gm_batch_status* summary);
/* XZ3IndexKeySpace.toIndexKey (idx/index/z3/XZ3IndexKeySpace.scala:60-95): bin + XZ3SFC(g, period).index
   of (envelope, offset) with the time from dtg (NULL / null slot -> 0) */
int gm_xz3_index_key_arrow(gm_ctx* ctx, const gm_geom_column* geom, const gm_time_column* dtg, int64_t n, int g,
                           int period, int lenient, int16_t* bin, int64_t* xz, uint8_t* status,
                           gm_batch_status* summary);
/* A point column as x / y device columns (null slots -> NaN): the adapter for every other entry */
int gm_arrow_points_to_columns(gm_ctx* ctx, const gm_geom_column* geom, int64_t n, double* x, double* y);
/* gm_pip_join_pred over an Arrow point column (null points never match): the direct pass reads the
   tuples in place */
int gm_pip_join_arrow(gm_ctx* ctx, const gm_pip_index* index, const gm_geom_column* points, int64_t n,
                      int64_t id_base, int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int64_t* n_pairs, int mode,
                      int predicate);
/* gm_pip_index_create_ex from an Arrow POLYGON or MULTIPOLYGON column given in HOST memory (the
   broadcast side of the join is collected on the host); a null slot is an empty polygon */
int gm_pip_index_create_arrow(gm_ctx* ctx, const gm_geom_column* polys, int32_t n, int cells_per_poly,
                              gm_pip_index** out);

/* ------------------------------------------------------------------ sorted key table */
/* The row-key prefix [shard?][bin BE16][z BE64] of Z3IndexKeySpace.toIndexKey (idx/index/z3/
   Z3IndexKeySpace.scala:81-92; ByteArrays.writeShort / writeLong, geomesa-utils/.../index/
   ByteArrays.scala:51,90-99) for n rows: out (device) gets n * key_len bytes, key_len = 11 with a
   shard column (device uint8, ShardStrategy.scala:75-80), 10 when shard = NULL.  The feature id
   the store appends after the prefix is the caller's. */
int gm_z3_key_bytes(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                    uint8_t* out);

/* The row-key prefix of the key spaces without a time bin: [shard?][z BE64] for Z2IndexKeySpace
   (idx/index/z2/Z2IndexKeySpace.scala:48-76) and XZ2IndexKeySpace (idx/index/z2/XZ2IndexKeySpace.scala:
   48-76, z = the XZ2 value): n * key_len bytes, key_len = 9 with a shard column, 8 without. */
int gm_z2_key_bytes(gm_ctx* ctx, const uint8_t* shard, const int64_t* z, int64_t n, uint8_t* out);

/* Sorts key columns into the table's row order -- the byte order of the row keys above: shard,
   then bin as an unsigned big-endian short, then z as an unsigned big-endian long (what Accumulo /
   HBase keep sorted).  Stable; perm_out[i] = the input row of table row i.  shard / shard_out may
   be NULL together (unsharded table); bin / bin_out may be NULL together (a key space without a time
   bin: Z2, XZ2).  n < 2^32.  Device temporaries: about 32.5 B per row (+ 4 B without a bin). */
int gm_sort_keys(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                 uint8_t* shard_out, int16_t* bin_out, int64_t* z_out, int64_t* perm_out);

/* Key-range partitioning of a table over GPUs (configs[2]: the table split into contiguous key ranges,
   one per rank, as a sorted store splits a table into tablets / regions, the shard prefix of
   ShardStrategy.scala:75-80 staying the key's first byte; it replaces the Spark shuffle of
   RelationUtils.scala:30-33, groupByKey(new IndexPartitioner(...))).  A key is the pair
   key_hi = shard << 16 | bin as u16 (0 <= key_hi < 2^24), key_lo = z as u64, compared unsigned
   lexicographically -- the byte order of [shard][bin BE16][z BE64].

   gm_key_sample: n_samples (<= 65536) keys of the UNSORTED columns at rows floor((2i+1) n / (2 n_samples))
   into key_hi / key_lo (host arrays).  Synchronises the context stream. */
int gm_key_sample(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n, int32_t n_samples,
                  uint64_t* key_hi, uint64_t* key_lo);
/* gm_key_partition: every row's destination d = the number of the n_split (< 256) ascending splitter keys
   (host arrays) <= its key; the rows are written grouped by destination (d ascending), keeping their
   input order within a destination, into shard_out / bin_out / z_out (device; shard and shard_out NULL
   together), with their source in ids_out (device, optional: ids[row] when ids (device) is given, else
   id_base + row) and / or rows_out (device, optional: the input row).  dest_counts (host, n_split + 1)
   receives each destination's row count; destination d's rows start at the sum of the counts before it.
   n < 2^32.  Synchronises the context stream. */
int gm_key_partition(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                     const uint64_t* split_hi, const uint64_t* split_lo, int32_t n_split, const int64_t* ids,
                     int64_t id_base, uint8_t* shard_out, int16_t* bin_out, int64_t* z_out, int64_t* ids_out,
                     uint32_t* rows_out, int64_t* dest_counts);

/* A scan range over the key prefix, inclusive at both ends in table order: what getRangeBytes
   makes of a ScanRange (idx/index/z3/Z3IndexKeySpace.scala:196-238), [toBytes(lo),
   toBytesFollowingPrefix(hi)) = every row whose [shard][bin][z] prefix lies in [lo, hi].
   BoundedRange(bin, lo, hi): bin_lo = bin_hi = bin; LowerBoundedRange: z_hi/bin_hi = all ones;
   UpperBoundedRange: bin_lo = z_lo = 0; UnboundedRange: both.  bin and z compare unsigned. */
typedef struct {
  int64_t z_lo;
  int64_t z_hi;
  int16_t bin_lo;
  int16_t bin_hi;
  uint8_t shard;       /* 0 for an unsharded table */
  uint8_t reserved[3];
} gm_key_range;

/* Seek-and-filter over a sorted table (gm_sort_keys order): every row inside any of the ranges
   (host array; sorted and merged here the way a BatchScanner merges overlapping ranges), then
   Z3Filter.inBounds on each (idx/filters/Z3Filter.scala:26-62, RowFilterIterator.scala:52-66) when
   filter_bytes (host, Z3Filter.serializeToBytes) is not NULL.  ids (device, optional) receives the
   matching rows in table order, mapped through perm (device, optional) to input rows.
   *n_match / *n_scanned (host) receive the match and candidate counts; GM_E_CAPACITY when the
   matches exceed ids_cap.  Synchronises the context stream. */
int gm_key_range_scan(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                      const gm_key_range* ranges, int64_t n_ranges, const uint8_t* filter_bytes, size_t filter_len,
                      const int64_t* perm, int64_t* ids, int64_t ids_cap, int64_t* n_match, int64_t* n_scanned);

/* The filters a table scan applies to its candidates (all optional; zero-initialise the struct):
   - the row filter the tablet server runs on each key (RowFilterIterator.scala:52-66): z3filter
     (host, Z3Filter.serializeToBytes: Z3Filter.inBounds on (bin, z), idx/filters/Z3Filter.scala:26-62)
     OR z2filter (host, Z2Filter.serializeToBytes: Z2Filter.inBounds on z, idx/filters/Z2Filter.scala:
     20-35), not both;
   - the full filter on the feature, which the XZ key spaces always apply (useFullFilter = true,
     XZ2IndexKeySpace.scala:122-125, XZ3IndexKeySpace.scala:247-250): with n_boxes > 0 the feature's
     envelope (xmin / ymin / xmax / ymax: device columns in INPUT order, reached through perm)
     intersects at least one of the boxes (host, n_boxes x (xmin, ymin, xmax, ymax); JTS
     Envelope.intersects, inclusive; a null envelope -- max < min -- never intersects), and with
     during != 0 the feature's dtg (t_ms: device, input order) lies in (t_lo, t_hi), exclusive
     (FastDuring, FastTemporalOperator.scala:116-129).  For a rectangular geometry the envelope test is
     GeoTools BBOX exactly; for other geometries it is BBOX's envelope pre-check (geometry-geometry
     relations are out of scope). */
typedef struct {
  const uint8_t* z3filter;
  size_t z3filter_len;
  const uint8_t* z2filter;
  size_t z2filter_len;
  const double* xmin;
  const double* ymin;
  const double* xmax;
  const double* ymax;
  const double* boxes;
  int32_t n_boxes;
  int32_t during;
  const int64_t* t_ms;
  int64_t t_lo;
  int64_t t_hi;
} gm_scan_filter;
/* Seek-and-filter over any sorted key table (gm_sort_keys order): Z3 and XZ3 tables ([shard][bin][z]),
   Z2 and XZ2 tables (bin = NULL: [shard][z]).  Every row inside any of the ranges (host array, merged as
   gm_key_range_scan merges them; for bin = NULL give bin_lo = bin_hi = 0, XZ2IndexKeySpace.getRangeBytes
   :104-120), then the filters of f (NULL = none).  ids (device, optional) receives the matching rows in
   table order, mapped through perm (device, optional) to input rows; *n_match / *n_scanned (host) the
   match and candidate counts; GM_E_CAPACITY when the matches exceed ids_cap.  Synchronises. */
int gm_table_scan(gm_ctx* ctx, const uint8_t* shard, const int16_t* bin, const int64_t* z, int64_t n,
                  const gm_key_range* ranges, int64_t n_ranges, const gm_scan_filter* f, const int64_t* perm,
                  int64_t* ids, int64_t ids_cap, int64_t* n_match, int64_t* n_scanned);

/* ------------------------------------------------------------------ legacy curves (reading / deleting old data) */
/* LegacyZ3SFC(period) (z3/curve/LegacyZ3SFC.scala:18-49): SemiNormalizedDimension lon/lat (2^21-1) and
   time (2^20-1) (NormalizedDimension.scala:83-97), ceil-based normalize, lenientIndex clamped from
   below only; LegacyYearZ3SFC (LegacyYearZ3SFC.scala:17-46): the 21-bit curve with the 52-week time
   max, offsets in (52 weeks, maxOffset(Year)] indexed as the max.  Device arrays, as gm_z3_index. */
#define GM_LEGACY_Z3 0
#define GM_LEGACY_YEAR_Z3 1
int gm_legacy_z3_index(gm_ctx* ctx, const double* x, const double* y, const int64_t* t, int64_t n, int curve,
                       int period, int lenient, int64_t* z, uint8_t* status, gm_batch_status* summary);
/* LegacyZ3SFC.invert = Z3SFC.invert with SemiNormalizedDimension.denormalize (curve GM_LEGACY_Z3 only) */
int gm_legacy_z3_invert(gm_ctx* ctx, const int64_t* z, int64_t n, int curve, int period, double* x, double* y,
                        int64_t* t);
/* LegacyZ2SFC (z3/curve/LegacyZ2SFC.scala:14-26): 2^31-1 semi-normalized lon/lat */
int gm_legacy_z2_index(gm_ctx* ctx, const double* x, const double* y, int64_t n, int lenient, int64_t* z,
                       uint8_t* status, gm_batch_status* summary);
int gm_legacy_z2_invert(gm_ctx* ctx, const int64_t* z, int64_t n, double* x, double* y);

/* ------------------------------------------------------------------ statistics */
/* Z3Histogram.observe / unobserve over a batch of point features (utils/stats/Z3Histogram.scala:101-128;
   a point's safeCentroid is the point): toKey (:80-86) = BinnedTime(period) + Z3SFC(period).index,
   lenient only for unobserve; a feature whose toKey throws is skipped (the Scala code logs a warning)
   and counted in tally[0].  The bin is LongBinning(length, (minZ, maxZ)).directIndex
   (utils/stats/BinnedArray.scala:185-201).  The histogram's binMap is the dense block
   counts[(timeBin - bin_lo) * length + i] (int64) for time bins bin_lo .. bin_lo + n_bins - 1 with
   present[timeBin - bin_lo] != 0 marking the bins binMap holds (observe sets it: getOrElseUpdate;
   unobserve only touches present bins: binMap.get(..).foreach).  Features whose time bin lies outside
   the window are counted in tally[1] and not added, so a caller can widen the window and re-run them.
   counts, present and tally (int64[2]) are device arrays and are accumulated into, never cleared; the
   call is asynchronous on the context stream. */
int gm_z3_histogram(gm_ctx* ctx, const double* x, const double* y, const int64_t* t_ms, int64_t n, int period,
                    int length, int unobserve, int bin_lo, int n_bins, uint8_t* present, int64_t* counts,
                    int64_t* tally);

/* ------------------------------------------------------------------ synthetic data (bench/tests) */
/* SplitMix64 keyed by (seed, index): lon U[lon0,lon1), lat U[lat0,lat1), t_ms U[t0,t1) */
int gm_gen_points(gm_ctx* ctx, uint64_t seed, int64_t n, int64_t index_base, double lon0, double lon1,
                  double lat0, double lat1, int64_t t0, int64_t t1, double* x, double* y, int64_t* t_ms);

#ifdef __cplusplus
}
#endif
#endif /* GEOMESA_HIP_H */
