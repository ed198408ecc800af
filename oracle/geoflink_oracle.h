/*
 * geoflink_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A plain-C CPU restatement of GeoFlink/SpatialFlink's window-evaluated spatial
 * query hot path (reference: marianaGarcez/SpatialFlink, Java 8 / Flink 1.9.1 /
 * JTS 1.16.1).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library.  The product (libgeoflink_hip.so) never links it.
 *
 * PARITY STATUS: "parity unpinned".  The reference ships no tests, golden vectors
 * or fixtures for this path, and it cannot run here (no
 * JDK, Flink or JTS jars; the JTS arithmetic it calls is a third-party dependency,
 * org.locationtech.jts:jts-core:1.16.1, pom.xml:59-63, absent from the reference
 * tree).  This restatement follows the reference files cited per function; the JTS
 * pieces (Coordinate.distance, Distance.pointToSegment, PointLocator /
 * RayCrossingCounter, Envelope.distance) restate JTS 1.16.1's published
 * algorithms.  It is cross-checked against an independent pure-Python restatement
 * (tests/golden/pyref.py) when the committed fixtures are generated.
 *
 * The operators are "reference-shaped": cell IDs are 10-char strings
 * (HelperClass.java:54-57,118-120), the guaranteed/candidate cell sets are string
 * hash sets built by the same loops as UniformGrid.java:165-229,368-445 (including
 * getIntCellIndices' substring parse, HelperClass.java:263-276), kNN runs per-cell
 * bounded max-heaps with java.util.PriorityQueue semantics and the windowAll merge
 * of KNNQuery.java:213-272 (objID-set bug included).
 */
#ifndef GEOFLINK_ORACLE_H
#define GEOFLINK_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* distance metric for JTS Coordinate.distance */
#define ORC_METRIC_SQRT  0   /* Math.sqrt(dx*dx + dy*dy) (default) */
#define ORC_METRIC_HYPOT 1   /* Math.hypot(dx, dy) == fdlibm e_hypot */

#define ORC_OK            0
#define ORC_ERR_CAPACITY -2
#define ORC_ERR_LAYERS   -5  /* reference: System.exit(1), UniformGrid.java:272-276 */
#define ORC_ERR_NPE      -6  /* reference: NullPointerException (KNNQuery.java:250-251 at k==1) */
#define ORC_ERR_ARG      -1

typedef struct {
  int32_t n;            /* numGridPartitions */
  double minX, maxX, minY, maxY;
  double cellLength;
} orc_grid;

/* UniformGrid(int uniformGridRows, minX, maxX, minY, maxY) -- UniformGrid.java:74-85 */
int orc_grid_make(int32_t n, double minX, double maxX, double minY, double maxY, orc_grid* g);

/* Java (int) cast of a double (JLS 5.1.3) */
int32_t orc_jint(double v);

/* HelperClass.assignGridCellID(Coordinate, UniformGrid) -- HelperClass.java:104-116 */
void orc_cell_of(const orc_grid* g, double x, double y, int32_t* cx, int32_t* cy);
/* HelperClass.generateCellIDStr / padLeadingZeroesToInt -- HelperClass.java:54-57,118-120; buf >= 32 */
void orc_cell_id(int32_t cx, int32_t cy, char* buf);
/* HelperClass.getIntCellIndices -- HelperClass.java:263-276 (substring(0,5) / substring(5)) */
void orc_parse_cell_id(const char* id, int32_t* cx, int32_t* cy);
void orc_assign_cells(const orc_grid* g, int64_t n, const double* x, const double* y,
                      int32_t* cx, int32_t* cy);

/* UniformGrid.getGuaranteedNeighboringLayers / getCandidateNeighboringLayers -- :428-445 */
int32_t orc_guaranteed_layers(const orc_grid* g, double r);
int32_t orc_candidate_layers(const orc_grid* g, double r);

/* JTS Coordinate.distance (metric selects sqrt-sum or fdlibm hypot) */
double orc_distance(double x1, double y1, double x2, double y2, int metric);
/* fdlibm e_hypot.c (what JDK 8 StrictMath.hypot / Math.hypot computes) */
double orc_hypot(double x, double y);

/* Guaranteed / candidate cell-set sizes for a single query cell (for tests) */
int64_t orc_gc_sets_point(const orc_grid* g, double r, int32_t qcx, int32_t qcy,
                          int32_t* g_cells /*2*capG or NULL*/, int64_t capG, int64_t* nG,
                          int32_t* c_cells /*2*capC or NULL*/, int64_t capC, int64_t* nC);

/* Window-based point-point range query, one window --
 * PointPointRangeQuery.java:111-187 (sets at :119-125, filter :135-140, apply :150-186).
 * Emits the multiset of point indices (approximate mode: C-cell points once per query
 * point) in input order.  Returns count (may exceed cap: only cap written). */
int64_t orc_range_pp(const orc_grid* g, int64_t n, const double* x, const double* y,
                     int32_t nq, const double* qx, const double* qy, double r,
                     int approximate, int metric, int64_t* out_idx, int64_t cap);

/* Polygons: CSR.  Polygon p owns rings [ring_off[p], ring_off[p+1]); ring j owns vertices
 * [vert_off[j], vert_off[j+1]) of (vx, vy).  Ring 0 of each polygon is the shell; rings
 * must be closed (first == last), as Polygon.createPolygon guarantees (Polygon.java:147-165). */
typedef struct {
  int32_t npoly;
  const int32_t* ring_off;
  const int32_t* vert_off;
  const double* vx;
  const double* vy;
} orc_polygons;

/* JTS Geometry.distance(point, polygon) -- DistanceFunctions.java:33-36 */
double orc_point_polygon_distance(double px, double py, const orc_polygons* P, int32_t p, int metric);
/* DistanceFunctions.getPointPolygonBBoxMinEuclideanDistance -- DistanceFunctions.java:150-200 */
double orc_point_bbox_distance(double px, double py, double x1, double y1, double x2, double y2);

/* Window-based point-polygon range query -- PointPolygonRangeQuery.java:134-205 */
int64_t orc_range_ppoly(const orc_grid* g, int64_t n, const double* x, const double* y,
                        const orc_polygons* P, double r, int approximate, int metric,
                        int64_t* out_idx, int64_t cap);

/* kNN, build contract: candidates = cell in C u G and d <= r; keep
 * the minimum-(d, idx) occurrence per objID; sort by (d, objID) ascending; first k.
 * Returns n_out (<= k) or a negative status. */
int32_t orc_knn_contract(const orc_grid* g, int64_t n, const double* x, const double* y,
                         const int64_t* objID, double qx, double qy, double r, int32_t k,
                         int metric, int64_t* out_objID, double* out_d, int64_t* out_idx);

/* kNN, reference-shaped: per-cell java.util.PriorityQueue (PointPointKNNQuery.java:159-192)
 * then kNNWinAllEvaluationPointStream (KNNQuery.java:213-272) incl. its objID-set bug.
 * Cells are visited in first-appearance order, points in arrival order.  Output is the
 * final queue in heap-array order.  Returns size, or ORC_ERR_NPE where Java throws. */
int32_t orc_knn_reference(const orc_grid* g, int64_t n, const double* x, const double* y,
                          const int64_t* objID, double qx, double qy, double r, int32_t k,
                          int metric, int64_t* out_objID, double* out_d, int64_t* out_idx);

/* orc_knn_reference on nthreads host threads, shaped as Flink runs the operator with
 * parallelism nthreads: source subtasks (contiguous point ranges: cell-ID string, HashSet C/G
 * filter, JTS distance) -> keyBy(gridID) hash shuffle -> key subtasks (per-cell bounded heaps)
 * -> one windowAll merge.  Same result as orc_knn_reference (the CPU baseline's all-core line). */
int32_t orc_knn_reference_mt(const orc_grid* g, int64_t n, const double* x, const double* y,
                             const int64_t* objID, double qx, double qy, double r, int32_t k,
                             int metric, int nthreads, int64_t* out_objID, double* out_d, int64_t* out_idx);

/* An optimised C kNN (build contract, = orc_knn_contract): OpenMP over point ranges, integer
 * Chebyshev cell test, squared-distance prefilter against each thread's running k-th distance,
 * per-thread bounded top-k-distinct heap, one merge.  The CPU baseline's second line. */
int32_t orc_knn_scan_omp(const orc_grid* g, int64_t n, const double* x, const double* y,
                         const int64_t* objID, double qx, double qy, double r, int32_t k,
                         int metric, int nthreads, int64_t* out_objID, double* out_d, int64_t* out_idx);

/* Window-based point-point join -- JoinQuery.java:73-90 + PointPointJoinQuery.java:124-183.
 * ugrid assigns ordinary points, qgrid assigns and replicates query points.
 * Writes pairs (ordinary idx, query idx) as out_pairs[2*i], out_pairs[2*i+1].
 * Returns pair count (may exceed cap) or ORC_ERR_LAYERS. */
int64_t orc_join_ppoly(const orc_grid* ugrid, const orc_grid* qgrid, int64_t no, const double* ox,
                       const double* oy, const orc_polygons* P, double r, int approximate, int metric,
                       int64_t* out_pairs, int64_t cap);
int64_t orc_join_ppoly_mt(const orc_grid* ugrid, const orc_grid* qgrid, int64_t no, const double* ox,
                          const double* oy, const orc_polygons* P, double r, int approximate, int metric,
                          int nthreads, int64_t* out_pairs, int64_t cap);
int64_t orc_join_pp(const orc_grid* ugrid, const orc_grid* qgrid,
                    int64_t no, const double* ox, const double* oy,
                    int64_t nq, const double* qx, const double* qy,
                    double r, int approximate, int metric, int64_t* out_pairs, int64_t cap);

/* HelperClass.generateQueryPolygons -- HelperClass.java:387-439.  Writes squares as
 * closed 5-vertex rings into vx/vy (5*cap each).  Returns polygon count (may exceed cap). */
int32_t orc_generate_query_polygons(int32_t numQueryPolygons, double minX, double minY,
                                    double maxX, double maxY, double* vx, double* vy, int32_t cap);

/* java.util.Random(seed); x = minX + nextDouble()*(maxX-minX), y likewise, per point
 * (cf. sncb/tests/SyntheticGpsSource.java:23,40-41) */
void orc_java_random_points(int64_t seed, int64_t n, double minX, double maxX,
                            double minY, double maxY, double* x, double* y);

/* PointPolygonKNNQuery.windowBased -- knn/PointPolygonKNNQuery.java:245-317, one query polygon
 * (P->npoly == 1), build contract as orc_knn_contract.  Returns the count or ORC_ERR_ARG. */
int32_t orc_knn_ppoly_contract(const orc_grid* g, int64_t n, const double* x, const double* y,
                               const int64_t* objID, const orc_polygons* P, double r, int32_t k,
                               int approximate, int metric, int64_t* out_objID, double* out_d,
                               int64_t* out_idx);
int32_t orc_knn_ppoly_mt(const orc_grid* g, int64_t n, const double* x, const double* y, const int64_t* objID,
                         const orc_polygons* P, double r, int32_t k, int approximate, int metric, int nthreads,
                         int64_t* out_objID, double* out_d, int64_t* out_idx);

/* Deserialization.CSVTSVToTSpatial.map over the lines of text (Deserialization.java:314-322):
 * want = csvTsvSchemaAttr (objID, time, x, y field indices).  Returns the line count (rows past
 * cap are not written); the first bad line and its kind (1 NumberFormatException, 2 hexadecimal
 * literal -- valid Java, value still written --, 3 missing field, 4 empty line) or -1. */
/* objID Strings: line i's String = oid[oid_off[i], oid_off[i+1]) (quotes removed, whitespace
 * kept); *oid_len = bytes needed (strings written only while they fit oid_cap). */
int64_t orc_csv_parse(const char* text, int64_t len, char delim, const int32_t* want, double* x, double* y,
                      char* oid, int64_t oid_cap, int64_t* oid_off, int64_t* oid_len, int64_t* ts, int64_t cap,
                      int64_t* bad_line, int32_t* bad_kind);

#ifdef __cplusplus
}
#endif

/* Multi-core CPU baselines (bench.py / tools/bench_workloads.py cpu_baseline lines): the
 * reference operators as Flink runs them with parallelism nthreads (source subtasks up to the
 * keyBy(gridID), a hash shuffle of the survivors, key subtasks running the apply) -- the same
 * results as orc_range_pp / orc_range_ppoly / orc_join_pp (indices ascending, pairs sorted). */
int64_t orc_range_pp_mt(const orc_grid* g, int64_t n, const double* x, const double* y, int32_t nq,
                        const double* qx, const double* qy, double r, int approximate, int metric, int nthreads,
                        int64_t* out_idx, int64_t cap);
int64_t orc_range_ppoly_mt(const orc_grid* g, int64_t n, const double* x, const double* y, const orc_polygons* P,
                           double r, int approximate, int metric, int nthreads, int64_t* out_idx, int64_t cap);
int64_t orc_join_pp_mt(const orc_grid* ugrid, const orc_grid* qgrid, int64_t no, const double* ox, const double* oy,
                       int64_t nq, const double* qx, const double* qy, double r, int approximate, int metric,
                       int nthreads, int64_t* out_pairs, int64_t cap);
int64_t orc_csv_parse_mt(const char* text, int64_t len, char delim, const int32_t* want, double* x, double* y,
                         int64_t* ts, int64_t cap, int nthreads, int64_t* bad_line, int32_t* bad_kind);
/* Optimised OpenMP lines (oracle/cpu_scan.c): integer cell classes instead of String keys,
 * per-thread outputs; the same results as the reference-shaped restatements. */
int64_t orc_range_pp_omp(const orc_grid* g, int64_t n, const double* x, const double* y, int32_t nq,
                         const double* qx, const double* qy, double r, int approximate, int metric, int nthreads,
                         int64_t* out_idx, int64_t cap);
int64_t orc_range_ppoly_omp(const orc_grid* g, int64_t n, const double* x, const double* y, const orc_polygons* P,
                            double r, int approximate, int metric, int nthreads, int64_t* out_idx, int64_t cap);
int64_t orc_join_pp_omp(const orc_grid* grid, int64_t no, const double* ox, const double* oy, int64_t nq,
                        const double* qx, const double* qy, double r, int metric, int nthreads, int64_t* out_pairs,
                        int64_t cap);
/* the same join's pair count, and *digest = sum mod 2^64 of fmix64(p << 32 | q) over its pairs */
int64_t orc_join_pp_omp_digest(const orc_grid* grid, int64_t no, const double* ox, const double* oy, int64_t nq,
                               const double* qx, const double* qy, double r, int metric, int nthreads,
                               uint64_t* digest);
#endif
