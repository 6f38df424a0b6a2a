/*
 * gm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of GeoMesa's spatio-temporal index-and-filter hot path
 * (liyq0307/geomesa, Scala).  It is the *checker* for the HIP product path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product library (geomesa_amd/lib/libgeomesa_hip.so) never links or calls it.
 *
 * Parity pinning: the restatement is checked against every known-answer test the
 * reference holds for this path; see tests/test_oracle_kats.py.
 * JTS (point-in-polygon) and GeoTools (strict BBOX edge inclusivity) semantics beyond the
 * axis-aligned box KATs are "parity unpinned" (no JVM in this image).
 *
 * Every function cites the reference file:line it restates; paths are relative to the
 * reference root and abbreviated:
 *   z3/  = geomesa-z3/src/main/scala/org/locationtech/geomesa/
 *   idx/ = geomesa-index-api/src/main/scala/org/locationtech/geomesa/index/
 */
#ifndef GM_ORACLE_H
#define GM_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-element status codes (mirror the JVM exception cases) */
#define GMO_OK            0
#define GMO_OUT_OF_BOUNDS 1   /* IllegalArgumentException from Z3SFC/Z2SFC/XZ require(...) */
#define GMO_BAD_TIME      2   /* BinnedTime require(...) : before 1970 or past the max date   */
#define GMO_UNORDERED     3   /* XZ require(xmin <= xmax ...) / ZRange require(min <= max)     */

/* TimePeriod (z3/curve/BinnedTime.scala:283-291) */
#define GMO_DAY   0
#define GMO_WEEK  1
#define GMO_MONTH 2
#define GMO_YEAR  3

typedef struct { int64_t lower, upper; int32_t contained; int32_t pad; } gmo_range;

/* ---- JVM conversions ---- */
int32_t gmo_d2i(double d);
int64_t gmo_d2l(double d);

/* ---- zorder/sfcurve ---- */
int64_t gmo_z3_split(int64_t v);
int32_t gmo_z3_combine(int64_t z);
int64_t gmo_z3_apply(int32_t x, int32_t y, int32_t t);
int64_t gmo_z2_split(int64_t v);
int32_t gmo_z2_combine(int64_t z);
int64_t gmo_z2_apply(int32_t x, int32_t y);
void    gmo_zdivide(int dims, int64_t p, int64_t rmin, int64_t rmax, int64_t* litmax, int64_t* bigmin);
int     gmo_zn_contains(int dims, int64_t rmin, int64_t rmax, int64_t value);
int     gmo_zn_overlaps(int dims, int64_t rmin, int64_t rmax, int64_t vmin, int64_t vmax);
void    gmo_longest_common_prefix(int dims, const int64_t* values, int n, int64_t* prefix, int* bits);
/* ZN.zranges: bounds = n pairs (min,max). returns count (<0 on error, -cap needed if cap too small) */
int64_t gmo_zranges(int dims, const int64_t* bounds, int nb, int precision, int max_ranges,
                    int max_recurse, gmo_range* out, int64_t cap);

/* ---- NormalizedDimension / BinnedTime ---- */
int32_t gmo_normalize(double min, double max, int precision, double x);
double  gmo_denormalize(double min, double max, int precision, int32_t i);
int64_t gmo_max_offset(int period);
int     gmo_binned_time(int period, int64_t ms, int16_t* bin, int64_t* offset);
int64_t gmo_binned_to_millis(int period, int16_t bin, int64_t offset);

/* ---- Z3SFC / Z2SFC ---- */
int     gmo_z3_index(int period, int precision, double x, double y, int64_t t, int lenient, int64_t* z);
void    gmo_z3_invert(int period, int precision, int64_t z, double* x, double* y, int64_t* t);
int     gmo_z2_index(int precision, double x, double y, int lenient, int64_t* z);
void    gmo_z2_invert(int precision, int64_t z, double* x, double* y);
/* Z3IndexKeySpace.toIndexKey (bin + z), batch */
void    gmo_z3_index_key_batch(int period, const double* x, const double* y, const int64_t* t_ms, int64_t n,
                               int lenient, int16_t* bin, int64_t* z, uint8_t* status);
/* legacy curves (LegacyZ3SFC / LegacyZ2SFC / LegacyYearZ3SFC) */
int     gmo_legacy_z3_index(int period, double x, double y, int64_t t, int lenient, int64_t* z);
void    gmo_legacy_z3_invert(int period, int64_t z, double* x, double* y, int64_t* t);
int     gmo_legacy_z2_index(double x, double y, int lenient, int64_t* z);
void    gmo_legacy_z2_invert(int64_t z, double* x, double* y);
int     gmo_legacy_year_z3_index(double x, double y, int64_t t, int lenient, int64_t* z);
/* Z3Histogram observe / unobserve (batch) and LongBinning.directIndex */
int     gmo_long_binning_index(int64_t min, int64_t max, int length, int64_t v);
void    gmo_z3_histogram(int period, const double* x, const double* y, const int64_t* t_ms, int64_t n, int length,
                         int unobserve, int bin_lo, int n_bins, uint8_t* present, int64_t* counts, int64_t* tally);
void    gmo_z2_index_batch(const double* x, const double* y, int64_t n, int lenient, int64_t* z, uint8_t* status);
void    gmo_z3_invert_batch(int period, const int64_t* z, int64_t n, double* x, double* y, int64_t* t);
void    gmo_z2_invert_batch(const int64_t* z, int64_t n, double* x, double* y);
/* xy = nxy*(xmin,ymin,xmax,ymax); t = nt*(tmin,tmax) */
int64_t gmo_z3_ranges(int period, int precision, const double* xy, int nxy, const int64_t* t, int nt,
                      int range_precision, int max_ranges, gmo_range* out, int64_t cap);
int64_t gmo_z2_ranges(int precision, const double* xy, int nxy, int range_precision, int max_ranges,
                      gmo_range* out, int64_t cap);

/* ---- XZ2SFC / XZ3SFC ---- */
int     gmo_xz2_index(int g, double xmin, double ymin, double xmax, double ymax, int lenient, int64_t* out);
int     gmo_xz3_index(int g, int period, double xmin, double ymin, double zmin, double xmax, double ymax,
                      double zmax, int lenient, int64_t* out);
void    gmo_xz2_index_batch(int g, const double* xmin, const double* ymin, const double* xmax, const double* ymax,
                            int64_t n, int lenient, int64_t* out, uint8_t* status);
void    gmo_xz3_index_batch(int g, int period, const double* xmin, const double* ymin, const double* zmin,
                            const double* xmax, const double* ymax, const double* zmax, int64_t n, int lenient,
                            int64_t* out, uint8_t* status);
int64_t gmo_xz2_ranges(int g, const double* q, int nq, int max_ranges, gmo_range* out, int64_t cap);
int64_t gmo_xz3_ranges(int g, int period, const double* q, int nq, int max_ranges, gmo_range* out, int64_t cap);

/* ---- Z3Filter / Z2Filter (serialized byte form, idx/filters/Z3Filter.scala:112-153) ---- */
int     gmo_z3filter_in_bounds(const uint8_t* filter, size_t len, const uint8_t* row, int offset);
int     gmo_z2filter_in_bounds(const uint8_t* filter, size_t len, const uint8_t* row, int offset);
/* columnar scan with bin restriction: returns match count, mask bit i set when row i passes */
int64_t gmo_z3filter_scan(const uint8_t* filter, size_t len, const int16_t* bin_ranges, int n_bin_ranges,
                          const int16_t* bin, const int64_t* z, int64_t n, uint8_t* match);
int64_t gmo_z2filter_scan(const uint8_t* filter, size_t len, const int64_t* z, int64_t n, uint8_t* match);
/* strict full filter: GeoTools BBOX (inclusive) AND FastDuring (exclusive, ms) */
int64_t gmo_strict_scan(const double* x, const double* y, const int64_t* t_ms, int64_t n,
                        const double* bbox, int has_during, int64_t during_lo, int64_t during_hi,
                        uint8_t* match);

/* ---- JTS-semantics point-in-polygon (st_contains(poly, point)) ---- */
typedef struct {
  int32_t n_polys;
  const int32_t* poly_part_off;   /* [n_polys+1] -> parts (polygon components) */
  const int32_t* part_ring_off;   /* [n_parts+1] -> rings; first ring of a part is the shell */
  const int32_t* ring_vert_off;   /* [n_rings+1] -> vertices; rings are closed (first == last) */
  const double*  vx;
  const double*  vy;
} gmo_polyset;

int     gmo_orientation_index(double p1x, double p1y, double p2x, double p2y, double qx, double qy);
/* 0 = EXTERIOR, 1 = BOUNDARY, 2 = INTERIOR (PointLocator with Mod-2 rule) */
int     gmo_locate(const gmo_polyset* ps, int poly, double px, double py);
int     gmo_contains(const gmo_polyset* ps, int poly, double px, double py);
int     gmo_intersects(const gmo_polyset* ps, int poly, double px, double py);
/* bbox AND during AND (OR over polygons of intersects (op 1) / contains (op 2)); NULL/0 = term absent */
int64_t gmo_query_scan(const double* x, const double* y, const int64_t* t_ms, int64_t n, const double* bbox,
                       int has_during, int64_t lo, int64_t hi, const gmo_polyset* ps, int op, uint8_t* match);
/* join: uniform-grid candidate generation + JTS contains. pairs written in (point, poly) order,
   sorted by point then poly. returns number of pairs (or -(needed) if cap too small). */
int64_t gmo_pip_join(const gmo_polyset* ps, const double* px, const double* py, int64_t n,
                     int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int nthreads);
int64_t gmo_pip_join_ex(const gmo_polyset* ps, const double* px, const double* py, int64_t n,
                        int64_t* pt_ids, int32_t* poly_ids, int64_t cap, int nthreads, int op, int64_t* cand_edges);

/* range decomposition work counter (per thread, read-and-reset) and the batch timing driver */
int64_t gmo_nodes_checked(void);
int     gmo_ranges_batch(int kind, int period, int g, const double* q, const int64_t* t, int64_t nq, int max_ranges,
                         int nthreads, int64_t* total_ranges, int64_t* total_nodes, int64_t* counts,
                         const int64_t* offsets, gmo_range* out);
#ifdef __cplusplus
}
#endif
#endif
