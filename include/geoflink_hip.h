/*
 * geoflink_hip.h -- C ABI of libgeoflink_hip.so, the MI355X (gfx950) window-evaluation
 * hot path of GeoFlink / SpatialFlink (reference: marianaGarcez/SpatialFlink).
 *
 * This is the drop-in boundary of BASELINE.json's north star: at each window trigger the
 * Java operators (UniformGrid, PointStream, RangeQuery, KNNQuery, JoinQuery) hand one
 * window's points across JNI as SoA buffers (x, y, objID, timestamp) and get the window's
 * result back.  Every entry point cites the reference code it replaces.  Plain C types only
 * (no torch, no C++); integer status codes, never exceptions or aborts across the boundary
 * (the reference's System.exit(1) becomes GF_ERR_LAYERS).  INTEGRATION.md shows the JNI
 * binding a maintainer adds on the Java side.
 *
 * Conventions
 *  - gf_points buffers are DEVICE pointers (HBM-resident windows).  x and y must be
 *    16-byte aligned (double2 loads).  gf_window_* upload host windows for callers that
 *    hold host buffers (JNI DirectByteBuffer / primitive arrays).
 *  - "async" calls only enqueue on the context's stream; "sync" calls return when results
 *    are on the host.
 *  - All arithmetic is IEEE binary64, round-to-nearest, no FMA contraction (Java never
 *    fuses), so cell IDs, range/join sets and kNN (objID, rank) lists match the reference
 *    restatement bit for bit.
 */
#ifndef GEOFLINK_HIP_H
#define GEOFLINK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GF_ABI_VERSION 2

/* status codes */
#define GF_OK             0
#define GF_ERR_ARG       -1  /* invalid argument (reference: IllegalArgumentException) */
#define GF_ERR_CAPACITY  -2  /* output capacity too small; the required count is returned */
#define GF_ERR_HIP       -3  /* HIP runtime error (see gf_ctx_last_error) */
#define GF_ERR_NOMEM     -4
#define GF_ERR_LAYERS    -5  /* candidate layers <= 0 where the reference calls System.exit(1)
                                (UniformGrid.java:272-276, JoinQuery.java:80) */
#define GF_ERR_ALIGN     -7  /* x / y not 16-byte aligned */
#define GF_ERR_COMM      -8  /* RCCL unavailable or a collective failed (see gf_comm_last_error) */

/* distance metric of JTS Coordinate.distance */
#define GF_METRIC_SQRT  0    /* Math.sqrt(dx*dx + dy*dy) -- default */
#define GF_METRIC_HYPOT 1    /* Math.hypot(dx, dy) (fdlibm e_hypot) */

/* kernel ids for gf_ctx_timing */
#define GF_K_KNN_SCAN    0
#define GF_K_KNN_SAMPLE  1
#define GF_K_KNN_SELECT  2
#define GF_K_RANGE_SCAN  3
#define GF_K_ASSIGN      4
#define GF_K_JOIN_PROBE  5
#define GF_K_RANGE_TEST  6  /* point-polygon join passes (the range plans' deferred tests run in the scan) */
#define GF_K_JOIN_BUCKET 7  /* ordinary-side bucketing of the join */
#define GF_K_KNN_MERGE   8  /* top-k record merges (shards, sliding-window panes) */
#define GF_K_CSV_PARSE   9  /* CSV ingest: the per-line parse kernel */
#define GF_K_BUCKET      10 /* K2 bucketing by cell (gf_bucket_by_cell) */
#define GF_K_JOIN_COMPACT 11 /* join: packing of the probe's task regions */
#define GF_K_COUNT       12

typedef struct gf_ctx gf_ctx;

/* UniformGrid(int n, minX, maxX, minY, maxY) -- UniformGrid.java:74-85 (value type) */
typedef struct {
  int32_t n;          /* numGridPartitions */
  int32_t reserved;
  double minX, maxX, minY, maxY;
  double cellLength;  /* (maxX - minX) / n, bounds NOT squared */
} gf_grid;

/* ---- objID keys ----------------------------------------------------------------------
 * The reference's objID is a String (Point.objID, Point.java:41-47; the CSV ingest keeps the
 * field as is, Deserialization.java:317 `String strOId`) and the kNN merge dedupes by
 * String.equals (KNNQuery.java:232-251).  gf_points.objID carries one int64 KEY per point,
 * injective over Strings:
 *   - a String that is exactly Long.toString(v) of a v in [-2^62, 2^62) -- "7", "-12"; not
 *     "007", "+7", " 7", "-0" -- has key v;
 *   - every other String has key INT64_MIN + id, its id in a gf_objid_dict -- assigned in first-
 *     occurrence order per batch, so keys never depend on scheduling.
 * Equal keys <=> equal Strings (keys of one dictionary).  The kNN contract's ties are broken by
 * key, so dictionary Strings order before numeric ones. */
#define GF_OBJID_NUMERIC_MIN (-(INT64_C(1) << 62))  /* keys below: dictionary Strings */
#define GF_OBJID_NUMERIC_END (INT64_C(1) << 62)     /* keys at or above: only GF_OBJID_NULL */
#define GF_OBJID_NULL INT64_MAX  /* a null objID (GeoJSON feature without the objID property) */
typedef struct gf_objid_dict gf_objid_dict;

/* One window of points as device SoA -- Point(objID, x, y, ts, uGrid), Point.java:91-100 */
typedef struct {
  const double* x;
  const double* y;
  const int64_t* objID;  /* objID keys (above); needed by kNN only */
  const int64_t* ts;     /* timeStampMillisec; unused by window evaluation */
  int64_t n;
} gf_points;

/* Query polygons (host CSR) -- Polygon(List<List<Coordinate>>, UniformGrid), Polygon.java:52-66.
 * Polygon p owns rings [ring_off[p], ring_off[p+1]); ring j owns vertices
 * [vert_off[j], vert_off[j+1]).  Ring 0 is the shell; rings are closed (first == last). */
typedef struct {
  int32_t npoly;
  const int32_t* ring_off;
  const int32_t* vert_off;
  const double* vx;
  const double* vy;
} gf_polygons;

/* ---- library / context ------------------------------------------------------------- */
int         gf_abi_version(void);
/* Build identity (no reference counterpart): the compile-time tuning / experiment defines every
 * translation unit of this library was built with ("" per unit for the product build), and the
 * GF_* run-time knobs set in the environment.  gf_build_is_product() == 1 iff no unit carries a
 * command-line define -- the smoke and the GPU suite require it, so an experiment build
 * (tools/build_exp.sh) can never be measured or tested as the product. */
const char* gf_build_info(void);
int         gf_build_is_product(void);
const char* gf_status_string(int status);
int         gf_device_count(int* n);
/* One context per calling thread / Flink subtask; binds `device`, owns scratch + a stream. */
int         gf_ctx_create(int device, gf_ctx** out);
void        gf_ctx_destroy(gf_ctx* ctx);
/* Borrow a caller stream (hipStream_t), e.g. torch's current stream; NULL = the HIP null
 * stream.  A new context starts on its own non-blocking stream (returned by gf_ctx_stream). */
int         gf_ctx_set_stream(gf_ctx* ctx, void* hip_stream);
void*       gf_ctx_stream(gf_ctx* ctx);
int         gf_ctx_synchronize(gf_ctx* ctx);
/* Make the context stream wait for everything enqueued so far on the context's other streams
 * (kNN pipeline depth >= 3 launches windows there); no-op when it has none.  Host does not block. */
int         gf_ctx_join(gf_ctx* ctx);
/* The converse: make the other streams wait for everything enqueued so far on the context
 * stream.  Call it after producing a window on the context stream and before a depth >= 3
 * gf_knn_enqueue of it (gf_window_points and gf_knn_run do it themselves). */
int         gf_ctx_fork(gf_ctx* ctx);
const char* gf_ctx_last_error(gf_ctx* ctx);
/* Context flags (testing / tuning).  GF_FLAG_JOIN_LEGACY: 1 = gf_join_pp probes the query
 * buckets from global memory in input order instead of the row-bucketed LDS path.
 * GF_FLAG_JOIN_COARSE: 1 = the row-bucketed path never takes its sub-cell (fine) variant.
 * GF_FLAG_GEOJSON_WALK: 1 = gf_geojson_parse takes the member-by-member walk on every line
 * (no one-pass locator); the results are the same.
 * GF_FLAG_JOIN_STREAM: 1 = gf_join_pp's fine path buckets only the query side and streams the
 * ordinary points in input order (an experiment the default path is measured against).
 * GF_FLAG_GEOJSON_WAVE: 1 = gf_geojson_parse locates members with the wave-per-line structural
 * scan (r06, measured slower: DESIGN.md §3 GeoJSON) instead of one line per lane; same results.
 * GF_FLAG_GEOJSON_CHECK: 1 = gf_geojson_parse runs the wave scan AND the lane locator on every
 * staged line and counts their differences (gf_geojson_check_counts); results as the default. */
#define GF_FLAG_JOIN_LEGACY 1
#define GF_FLAG_JOIN_COARSE 2
#define GF_FLAG_GEOJSON_WALK 4
#define GF_FLAG_JOIN_STREAM 8
#define GF_FLAG_GEOJSON_WAVE 16
#define GF_FLAG_GEOJSON_CHECK 32
int gf_ctx_set_flag(gf_ctx* ctx, int flag, int value);
/* GF_FLAG_GEOJSON_CHECK's counts since the last read (then zeroed), after a sync: out[0] lines
 * both passed with the same member notes, out[1] the wave scan passed and the lane locator did not,
 * out[2] both passed with different notes, out[3] the lane locator passed and the wave scan did not
 * (a byte >= 0x80 sends a line to the walk).  out[1] and out[2] are defects. */
int gf_geojson_check_counts(gf_ctx* ctx, unsigned long long out[4]);

/* Record HIP events around launches of the kernels in `mask` (bit 1 << GF_K_*; 0 = off). */
int         gf_ctx_set_timing(gf_ctx* ctx, int mask);
/* Time only every period-th launch of each kernel (fewer events in a hot loop); default 1. */
int         gf_ctx_set_timing_period(gf_ctx* ctx, int period);
/* Sync, then return the summed kernel time (ms) and launch count for kernel_id; resets it. */
int         gf_ctx_timing(gf_ctx* ctx, int kernel_id, double* total_ms, int64_t* launches);

/* ---- grid / cell IDs (host) -------------------------------------------------------- */
int gf_grid_make(int32_t n, double minX, double maxX, double minY, double maxY, gf_grid* out);
/* getGuaranteedNeighboringLayers / getCandidateNeighboringLayers -- UniformGrid.java:428-445 */
int gf_grid_layers(const gf_grid* g, double r, int32_t* guaranteed, int32_t* candidate);
/* assignGridCellID(Coordinate) -- HelperClass.java:104-116 (host scalar form) */
int gf_cell_of(const gf_grid* g, double x, double y, int32_t* cx, int32_t* cy);
/* "%05d%05d" -- HelperClass.java:54-57,118-120; returns GF_ERR_CAPACITY if cap too small */
int gf_format_cell_id(int32_t cx, int32_t cy, char* buf, int32_t cap);
/* getIntCellIndices -- HelperClass.java:263-276 */
int gf_parse_cell_id(const char* id, int32_t* cx, int32_t* cy);

/* ---- K1: grid-cell assignment (async) -----------------------------------------------
 * Replaces HelperClass.assignGridCellID per point at ingest (Point.java:98).  cx/cy are
 * device int32[n]: cx = (int)Math.floor((x - minX)/cellLength), Java (int) saturation. */
int gf_assign_cells(gf_ctx* ctx, const gf_grid* g, const gf_points* pts, int32_t* cx, int32_t* cy);

/* ---- K2: bucketing by cell (async) -- the keyBy(gridID) shuffle (PointPointRangeQuery.java:144-148)
 * perm: device uint32[n], point indices grouped by cell; cell_start: device uint32[n*n + 2],
 * bucket b = valid cell cy*n + cx, bucket n*n = out-of-grid points: bucket b is
 * perm[cell_start[b] .. cell_start[b+1]).  Stable: inside a bucket the points keep their input
 * order (Flink's per-key window buffer iterates in arrival order), so the result is unique. */
int gf_bucket_by_cell(gf_ctx* ctx, const gf_grid* g, const gf_points* pts, uint32_t* perm,
                      uint32_t* cell_start);

/* ---- multi-GPU routing of an arriving window (async) ---------------------------------
 * The window's points partitioned by owning GPU: band b owns cell columns [band_lo[b],
 * band_lo[b+1]) (columns left of band_lo[1] -- out-of-grid ones too -- belong to band 0, those
 * right of the last start to the last band; NaN x counts as column 0).  perm: device
 * uint32[n], every band's points in arrival order; offsets: device uint32[nbands + 1], band b =
 * perm[offsets[b] .. offsets[b+1]).  One stable radix pass over the band keys (K1 + K2), the
 * keyBy(gridID) shuffle across ranks (PointPointRangeQuery.java:144-148).  nbands <= 64. */
int gf_shard_by_columns(gf_ctx* ctx, const gf_grid* g, const gf_points* pts, int32_t nbands, const int32_t* band_lo,
                        uint32_t* perm, uint32_t* offsets);
/* A band's SoA slice: out[i] = in[perm[begin + i]], i < end - begin, for the columns given
 * (device buffers; x, y, objID, ts may each be null). */
int gf_gather_points(gf_ctx* ctx, const gf_points* pts, const uint32_t* perm, int64_t begin, int64_t end, double* x,
                     double* y, int64_t* objID, int64_t* ts);

/* ---- range queries ----------------------------------------------------------------- */
typedef struct gf_range_plan gf_range_plan;
/* PointPointRangeQuery.run(stream, Set<Point> queryPoints, r) -- guaranteed / candidate cell
 * sets built once (PointPointRangeQuery.java:119-125); qx/qy host arrays. */
int  gf_range_pp_plan_create(gf_ctx* ctx, const gf_grid* g, const double* qx, const double* qy,
                             int32_t nq, double r, int approximate, int metric, gf_range_plan** out);
/* PointPolygonRangeQuery.run(stream, Set<Polygon>, r) -- PointPolygonRangeQuery.java:138-147 */
int  gf_range_ppoly_plan_create(gf_ctx* ctx, const gf_grid* g, const gf_polygons* polys, double r,
                                int approximate, int metric, gf_range_plan** out);
void gf_range_plan_destroy(gf_range_plan* plan);
/* Window apply (PointPointRangeQuery.java:150-186 / PointPolygonRangeQuery.java:170-204), async.
 * bitmap: device uint64[(n+63)/64], bit i = point i emitted.  multi_bitmap (nullable): bit i =
 * point i emitted once per query point (approximate point-point, C cells).  counts: device
 * int64[2] = {points emitted, size of the emitted multiset}, summed by the last block of the
 * window's last kernel (no extra launch). */
int  gf_range_run(gf_range_plan* plan, const gf_points* pts, uint64_t* bitmap,
                  uint64_t* multi_bitmap, int64_t* counts);
/* Up to 16 windows of one plan in ONE launch (window w = pts[w], its bitmap bitmaps[w] and
 * counts[w] as gf_range_run; no multiplicity bitmap), plus -- idx non-null -- every window's
 * ascending index list in one more launch (idx[w] of capacity idx_cap[w], its length to
 * idx_count[w], as gf_bitmap_to_indices_async).  Async.  For windows that are available together
 * (a catch-up, several keys): small windows stop paying a launch each (PointPointRangeQuery.java:
 * 150-186 per window). */
int  gf_range_run_batch(gf_range_plan* plan, int32_t nwin, const gf_points* pts, uint64_t* const* bitmaps,
                        int64_t* const* counts, uint32_t* const* idx, const int64_t* idx_cap, int64_t* const* idx_count);
/* Plan diagnostics: in-grid cells by class (none / candidate / guaranteed / candidate cells
 * accepted untested because closed rectangles cover them); any pointer may be null. */
int  gf_range_plan_stats(const gf_range_plan* plan, int64_t* none_cells, int64_t* candidate_cells,
                         int64_t* guaranteed_cells, int64_t* inside_cells);
/* Tuning: scan blocks (0 = auto, <= 8 per CU); candidate tests: 0 auto, 1 inline in the scan,
 * 2 deferred (each scan block tests the candidate-cell points it queued at its end), 3 deferred
 * with the span prefilter (the scan only rules out points outside the class spans; every other
 * point is classified by the table at the block's end) -- table modes. */
int  gf_range_plan_set_tuning(gf_range_plan* plan, int32_t scan_blocks, int32_t defer_mode);
/* Testing: the deferred candidate tests at each scan block's end run on the first `lanes` lanes of
 * every wave only (1..64; 0 = all, the default).  Results are identical for any value: the drain
 * takes its points from a block cursor with whatever lanes are active (tests/test_gpu_parity.py). */
int  gf_range_plan_set_drain_lanes(gf_range_plan* plan, int32_t lanes);
/* Sync: selection bitmap -> ascending point indices (device uint32[cap]). */
int  gf_bitmap_to_indices(gf_ctx* ctx, const uint64_t* bitmap, int64_t n, uint32_t* idx,
                          int64_t cap, int64_t* count);
/* Async, one launch: the same indices (those past cap are not written) and their count into
 * device int64 *count -- enqueue it after gf_range_run so a window's step ends with the index
 * list the Java collector emits (PointPointRangeQuery.java:150-186) without a host sync. */
int  gf_bitmap_to_indices_async(gf_ctx* ctx, const uint64_t* bitmap, int64_t n, uint32_t* idx,
                                int64_t cap, int64_t* count);

/* ---- kNN ---------------------------------------------------------------------------- */
typedef struct gf_knn_plan gf_knn_plan;
/* PointPointKNNQuery.run(stream, queryPoint, r, k) -- PointPointKNNQuery.java:33,132-150 */
int    gf_knn_pp_plan_create(gf_ctx* ctx, const gf_grid* g, double qx, double qy, double r,
                             int32_t k, int metric, gf_knn_plan** out);   /* 1 <= k <= 2^24 */
/* k <= 512: sample -> scan -> one-block select (pipeline depths 1..3).  k > 512 (the
 * reference's PriorityQueue takes any k, KNNQuery.java:216): every candidate within r is kept
 * and the record comes from two stable device radix sorts of them ((objID, d, idx) -> first of
 * each objID -> (d, objID, idx)); the passes are sized by the window and bounded by the counts
 * on the device, so the enqueue never synchronizes and windows queue back to back at any
 * pipeline depth (each record complete in stream order); the sliding engine and
 * gf_knn_merge_dev(_batch) take records of any k.  The exact re-evaluation of a flagged window
 * (gf_knn_decode) takes the same sorted path. */
/* PointPolygonKNNQuery.run(stream, queryPolygon, r, k) -- knn/PointPolygonKNNQuery.java:245-317:
 * kNN of the window's points to ONE query polygon (polys->npoly == 1): candidates have their cell
 * in C u G of the polygon's bbox cells and d <= r, d = JTS point-polygon distance (0 inside) or,
 * approximate, DistanceFunctions.getPointPolygonBBoxMinEuclideanDistance.  Same records, decode
 * and contract as point queries ((d, objID) order, one entry per objID); pipeline depth <= 2. */
int    gf_knn_ppoly_plan_create(gf_ctx* ctx, const gf_grid* g, const gf_polygons* polys, double r, int32_t k,
                                int approximate, int metric, gf_knn_plan** out);
void   gf_knn_plan_destroy(gf_knn_plan* plan);
/* Candidate-buffer capacity (entries); default 1<<20.  Small values force the exact fallback. */
int    gf_knn_plan_set_capacity(gf_knn_plan* plan, int64_t cap);
/* Scan-kernel tuning: grid blocks (0 = auto), point pairs per lane per iteration (1..8),
 * nontemporal loads (0/1).  Results never depend on it. */
int    gf_knn_plan_set_tuning(gf_knn_plan* plan, int32_t scan_blocks, int32_t unroll, int32_t nontemporal);
/* Continuous-query threshold hint (default on): each window stores 2 x its k-th distance and
 * the next window scans only below it (still verified: >= k distinct objIDs or re-evaluate). */
int    gf_knn_plan_set_hint(gf_knn_plan* plan, int enable);
/* Offset added to the window-local point index in results (a shard's first global index). */
int    gf_knn_plan_set_index_base(gf_knn_plan* plan, int64_t base);
/* Continuous-query pipeline.  depth 1 (default): each enqueue runs sample -> scan -> select,
 * stream-ordered.  depth 2 (k <= 256; larger k below): ONE fused launch per window -- blocks 1.. scan window i
 * with the threshold hint left by window i-2 (two device lanes), block 0 runs window i-1's
 * select meanwhile.  Window i's record is therefore written by the NEXT enqueue on the plan,
 * or by gf_knn_plan_flush (stream-ordered on the context stream).  No sample kernel: a cold
 * or failed hint flags the window (status 1, re-evaluated exactly by gf_knn_decode) and the
 * threshold adapts (shrinks after an overflow, doubles when fewer than k lie below it).
 * depth d = 3 or 4 (k <= 256): S = d - 1 streams (the context stream + S - 1 non-blocking ones);
 * window i launches on stream i % S, scans lane i % 2S and selects window i - S -- the previous
 * launch on the same stream -- in block 0, so S launches are in flight and every dependency stays
 * stream-ordered.  Polygon plans: the same, with each window's refine after its prefilter launch.
 * Window buffers must be complete before their enqueue: no cross-stream wait is inserted for them
 * (gf_ctx_fork after producing one on the context stream); gf_knn_plan_flush joins the other
 * streams back.  k in (256, 512] at depth >= 2: the select needs the standalone kernel's sort
 * area, so it is not fused: each window runs [sample] + scan + select on its lane, its record
 * complete in stream order; depth d >= 3 spreads windows over S streams, one lane each.  k > 512:
 * see above.  The sliding engine rejects depth > 2.  Results are identical at every depth. */
int    gf_knn_plan_set_pipeline(gf_knn_plan* plan, int depth);
int    gf_knn_plan_flush(gf_knn_plan* plan);
/* Result record: gf_knn_header followed by double dist[k], int64 objID[k], int64 idx[k]. */
typedef struct {
  int32_t status;        /* 0 = final; 1 = needs the exact fallback (see gf_knn_decode);
                            2 = a GF_MERGE_FOREIGN_KEYS merge met dictionary objID keys */
  int32_t n;             /* entries (<= k) */
  int32_t k;
  int32_t flags;
  int64_t candidates;    /* candidates appended by the scan */
  double threshold;      /* distance threshold the scan used */
} gf_knn_header;
size_t gf_knn_result_bytes(int32_t k);
/* Per-cell heaps + windowAll merge (PointPointKNNQuery.java:159-200, KNNQuery.java:213-272),
 * async: writes one result record into device memory `result`. */
int    gf_knn_enqueue(gf_knn_plan* plan, const gf_points* pts, void* result);
/* Sync: decode a host copy of the record; if it asks for the exact fallback, run it on pts.
 * Outputs sorted ascending by (dist, objID): rank = position. */
int    gf_knn_decode(gf_knn_plan* plan, const gf_points* pts, const void* result_host,
                     int64_t* objID, double* dist, int64_t* idx, int32_t* n_out);
/* Sync convenience: enqueue + copy + decode. */
int    gf_knn_run(gf_knn_plan* plan, const gf_points* pts, int64_t* objID, double* dist,
                  int64_t* idx, int32_t* n_out);
/* Merge per-shard top-k records (device, `nrec` <= 64 contiguous records of
 * gf_knn_result_bytes(k)) into one record (async) -- the windowAll funnel across GPUs after
 * an RCCL all-gather.  `result` may be device memory or gf_pinned_alloc memory.  Any k
 * (1 <= k <= 2^24): k <= 512 in one 256-thread block's LDS; larger k ranks every entry by binary
 * searches in the other records (each is sorted by (d, objID, idx)) and dedupes objIDs through
 * a hash table in the context's scratch, one 1024-thread block per window. */
int    gf_knn_merge_dev(gf_ctx* ctx, int32_t k, const void* records, int32_t nrec, void* result);
/* Batched: nwin windows in one launch (one block each), so one RCCL all-gather can carry the
 * records of several windows.  layout GF_MERGE_SHARD_MAJOR: record (shard s, window w) at
 * index s*nwin + w (an all-gather of each rank's nwin consecutive records);
 * GF_MERGE_WINDOW_MAJOR: at index w*nrec + s.  `results` receives nwin consecutive records.
 * layout | GF_MERGE_FOREIGN_KEYS: the records come from other contexts (an all-gather across
 * ranks).  Dictionary objID keys (below GF_OBJID_NUMERIC_MIN, GF_OBJID_NULL aside) are ids in
 * their own context's gf_objid_dict, so keys of different ranks cannot be compared or deduped:
 * a window holding one gets status 2 (GF_KNN_STATUS_FOREIGN_KEYS) and no entries -- merge such
 * windows by their Strings instead (gf_knn_attach_strings + gf_knn_merge_dev_strings below).
 * Canonical decimal objIDs are their values and merge across ranks. */
#define GF_MERGE_SHARD_MAJOR  0
#define GF_MERGE_WINDOW_MAJOR 1
#define GF_MERGE_FOREIGN_KEYS 0x100
#define GF_KNN_STATUS_FOREIGN_KEYS 2
int    gf_knn_merge_dev_batch(gf_ctx* ctx, int32_t k, const void* records, int32_t nrec, int32_t nwin,
                              int32_t layout, void* results);
/* ---- String objIDs across ranks (KNNQuery.java:232-251 dedupes by String.equals; MN_Q1.java:52
 * feeds gps.deviceId Strings).  A dictionary key is an id in its own rank's dictionary, so the
 * records travel with their Strings: a STRING RECORD is a kNN record followed by a sidecar
 * {int32 status, int32 n, int64 nbytes, uint32 off[k+1] (8-aligned), bytes[cap_bytes]} holding
 * the String of every dictionary objID of the record (entry i = bytes[off[i], off[i+1]), empty for
 * canonical decimal / null keys); sidecar status 1 = the Strings needed more than cap_bytes.
 *   rank r: gf_knn_attach_strings(its dictionary, its records) -> all-gather the string records
 *   -> gf_knn_merge_dev_strings on every rank -> the same merged string record everywhere.
 * The merge orders by (d, String, idx) -- dictionary Strings by their bytes (unsigned, a prefix
 * first) and before canonical decimals, decimals by value (null last) -- and keeps the first
 * entry of every String: rank independent.  (One rank's own select orders tied distances by
 * dictionary id; the cross-rank order differs from it only between different Strings at exactly
 * equal distances.)  The merged record's dictionary keys are the source ranks' and mean nothing
 * elsewhere: read its Strings with gf_knn_string_record_decode.  A flagged input record (status 1)
 * gives a flagged merged record (status 1, no entries: re-evaluate the shard exactly and exchange
 * again, as for gf_knn_exchange_batch); an input whose Strings did not fit its sidecar gives
 * status 2 (GF_KNN_STATUS_FOREIGN_KEYS, no entries: retry with a larger cap_bytes). */
size_t gf_knn_string_record_bytes(int32_t k, int64_t cap_bytes);
/* Async: nrec consecutive records (gf_knn_result_bytes(k) apart, device or pinned memory) ->
 * nrec consecutive string records (gf_knn_string_record_bytes(k, cap_bytes) apart) with the
 * Strings of their dictionary keys read from `dict` on the device. */
int gf_knn_attach_strings(gf_objid_dict* dict, int32_t k, const void* records, int32_t nrec, int64_t cap_bytes,
                          void* out);
/* Async: as gf_knn_merge_dev_batch (layouts, nrec <= 64, one block per window, any k) over string
 * records; results = nwin consecutive merged string records. */
int gf_knn_merge_dev_strings(gf_ctx* ctx, int32_t k, int64_t cap_bytes, const void* records, int32_t nrec,
                             int32_t nwin, int32_t layout, void* results);
/* Host: decode a host copy of a string record: *status (0 ok, else the record's / 2), entries
 * (objID keys, dist, idx; any may be null) and their Strings, String j = buf[offs[j], offs[j+1])
 * (Long.toString for canonical decimal keys, empty for null); GF_ERR_CAPACITY when buf_cap is too
 * small (offs[n] = the bytes needed). */
int gf_knn_string_record_decode(const void* record, int32_t k, int64_t cap_bytes, int32_t* status, int64_t* objID,
                                double* dist, int64_t* idx, char* buf, int64_t buf_cap, int64_t* offs, int32_t* n_out);
/* Host merge of per-shard sorted lists: top-k distinct objIDs by (dist, objID). */
int    gf_knn_merge_host(int32_t k, int32_t nlists, const int32_t* counts, const int64_t* objID,
                         const double* dist, const int64_t* idx, int64_t* out_objID,
                         double* out_dist, int64_t* out_idx, int32_t* n_out);

/* ---- multi-GPU: RCCL communicators and the kNN record exchange --------------------------------
 * The windowAll funnel across GPUs (PointPointKNNQuery.java:198-200 -> KNNQuery.java:213-272):
 * each GPU evaluates its cell-column band of the window (gf_shard_by_columns routes an arriving
 * window) into a top-k record; the exchange all-gathers every rank's records over xGMI (RCCL
 * ncclAllGather on the context's stream) and merges them on the device into the SAME record on
 * every rank (gf_knn_merge_dev_batch, shard-major; with > 1 rank GF_MERGE_FOREIGN_KEYS).  RCCL is
 * opened on first use (dlopen librccl.so.1; a process already holding it shares that copy).
 *   one process per GPU:  rank 0 gf_comm_unique_id -> broadcast the 128 bytes over the job's own
 *                         control plane -> every rank gf_comm_create(id, nranks, rank, device)
 *                         (ncclCommInitRank; blocks until all ranks joined);
 *   one process, N GPUs:  gf_comm_create_all(N, devices, comms) (ncclCommInitAll) -- then one
 *                         thread per GPU calls gf_knn_exchange_batch on its own comm, or one
 *                         thread drives all of them with gf_knn_exchange_group.
 * A communicator's exchanges must be enqueued on one stream (its gather buffer is reused in
 * stream order).  Every rank must call the exchange with the same k and nwin, in the same order.
 * Input records must be final (status 0): a flagged record (status 1) makes the merged record
 * flagged on every rank -- re-evaluate the shard exactly (gf_knn_decode) and exchange again. */
#define GF_COMM_ID_BYTES 128
typedef struct gf_comm gf_comm;
int  gf_comm_available(void);               /* 1 when librccl.so.1 loads and has every entry used */
int  gf_comm_unique_id(uint8_t* id);        /* id[GF_COMM_ID_BYTES] (ncclGetUniqueId), on one rank */
int  gf_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int device, gf_comm** out);
int  gf_comm_create_all(int32_t ndev, const int* devices, gf_comm** out /* [ndev] */);
void gf_comm_destroy(gf_comm* comm);        /* drains the device first */
int  gf_comm_info(const gf_comm* comm, int32_t* nranks, int32_t* rank, int* device);
const char* gf_comm_last_error(const gf_comm* comm);  /* comm == NULL: why this thread's last unique-id /
                                                      create call failed, else why RCCL did not load */
int  gf_comm_check(gf_comm* comm);          /* GF_ERR_COMM on an asynchronous RCCL error */
/* Async: this rank's nwin consecutive device records (gf_knn_result_bytes(k) apart; ctx's device
 * == the comm's) -> `merged` = nwin consecutive merged records (device or mapped pinned memory),
 * identical on every rank.  One all-gather + one merge launch for all nwin windows. */
int gf_knn_exchange_batch(gf_comm* comm, gf_ctx* ctx, int32_t k, const void* records, int32_t nwin, void* merged);
/* Async, String objIDs: the records' dictionary Strings attached from `dict` (on dict's context,
 * gf_knn_attach_strings), the string records all-gathered, merged by String
 * (gf_knn_merge_dev_strings) -> nwin merged string records (gf_knn_string_record_bytes apart). */
int gf_knn_exchange_strings_batch(gf_comm* comm, gf_objid_dict* dict, int32_t k, int64_t cap_bytes,
                                  const void* records, int32_t nwin, void* merged);
/* Async, one thread driving n communicators of one clique (gf_comm_create_all): the n
 * all-gathers as one RCCL group, then the n merges (comms[i] with ctxs[i], records[i], merged[i]).
 * comms must be the WHOLE clique (n == its size, each rank once; GF_ERR_ARG otherwise), checked
 * with every other argument before the group starts.  Should RCCL still fail inside the group,
 * the clique is aborted (ncclCommAbort: no all-gather is left waiting for a peer) and every later
 * call on those communicators returns GF_ERR_COMM; destroy them and create a new clique. */
int gf_knn_exchange_group(int32_t n, gf_comm* const* comms, gf_ctx* const* ctxs, int32_t k,
                          const void* const* records, int32_t nwin, void* const* merged);

/* ---- sliding-window kNN: pane engine ------------------------------------------------
 * PointPointKNNQuery.windowBased with SlidingProcessingTimeWindows.of(size, slide)
 * (PointPointKNNQuery.java:158,198-200; KNNQuery.java:213-272).  The reference re-evaluates
 * every window from scratch (each point size/slide times); here the stream is cut into panes
 * of gcd(size, slide) ms, each pane is evaluated ONCE on `plan` into a device record ring, and
 * a window's record is the top-k-distinct merge of its panes' records -- identical to
 * evaluating the window whole.  Pane p holds timestamps [p*pane_ms, (p+1)*pane_ms) (Flink
 * window assignment, offset 0); window [s, s + size), s a multiple of slide, closes with the
 * pane ending at s + size, and fires only if it holds a point.  Result idx = the point's position
 * in the pushed stream (panes concatenated in push order). */
typedef struct gf_knn_sliding gf_knn_sliding;
/* size / gcd(size, slide) <= 64; any k (k > 512: pane records from the sorted path, merged by
 * rank).  The plan's pipeline depth applies (depth 2: one fused launch per pane for k <= 256). */
int  gf_knn_sliding_create(gf_knn_plan* plan, int64_t size_ms, int64_t slide_ms, gf_knn_sliding** out);
void gf_knn_sliding_destroy(gf_knn_sliding* s);
/* pane length, panes per window / per slide, and how many of the latest panes the engine keeps
 * (their device buffers are borrowed and must stay valid while in the ring) */
int  gf_knn_sliding_geometry(const gf_knn_sliding* s, int64_t* pane_ms, int32_t* panes_per_window,
                             int32_t* panes_per_slide, int32_t* ring_panes);
/* Async.  Push pane `pane_index` (consecutive indices; an empty pane is pushed with n = 0).  If
 * a window closes with it, *closed = 1, *window_end = its end (ms), and its record is written
 * to window_result (device or gf_pinned_alloc memory) -- at depth 2 by the next push or flush. */
int  gf_knn_sliding_push(gf_knn_sliding* s, int64_t pane_index, const gf_points* pane, void* window_result,
                         int32_t* closed, int64_t* window_end);
int  gf_knn_sliding_flush(gf_knn_sliding* s);
/* Sync: decode a host copy of a window record; a flagged record (a pane needed the exact
 * fallback) is re-evaluated pane by pane (the panes must still be in the ring). */
int  gf_knn_sliding_decode(gf_knn_sliding* s, int64_t window_end, const void* result_host, int64_t* objID,
                           double* dist, int64_t* idx, int32_t* n_out);

/* ---- sliding range: the pane engine for PointPointRangeQuery / PointPolygonRangeQuery under
 * SlidingProcessingTimeWindows.of(size, slide) (PointPointRangeQuery.java:149-186,
 * PointPolygonRangeQuery.java:170-204).  Each pane (gcd(size, slide) ms, as gf_knn_sliding) is
 * evaluated ONCE on `plan` -- gf_range_run into a device pane bitmap, compacted on the device into
 * the pane's index list -- and a closed window's emitted points are its panes' lists
 * concatenated: identical to evaluating the window whole (each point's test is independent).
 * Window indices are window-local: positions in the window's panes concatenated in push order,
 * ascending, each emitted point once (approximate multi-query multiplicity: gf_range_run). */
typedef struct gf_range_sliding gf_range_sliding;
/* size / gcd(size, slide) <= 64; plan: gf_range_pp_plan_create / gf_range_ppoly_plan_create */
int  gf_range_sliding_create(gf_range_plan* plan, int64_t size_ms, int64_t slide_ms, gf_range_sliding** out);
void gf_range_sliding_destroy(gf_range_sliding* s);
int  gf_range_sliding_geometry(const gf_range_sliding* s, int64_t* pane_ms, int32_t* panes_per_window,
                               int32_t* panes_per_slide);
/* Async.  Push pane `pane_index` (consecutive indices; an empty pane with n = 0; the pane's
 * device points must stay valid until the context stream has passed this call).  If a window
 * closes with it and holds a point: *closed = 1, *window_end = its end (ms), *window_n = its
 * points, and the stream writes the window's index list to idx (device or pinned uint32[cap])
 * and its length to *count (device or pinned int64).  cap < *window_n: GF_ERR_CAPACITY with
 * nothing enqueued (push the same pane again with a larger idx). */
int  gf_range_sliding_push(gf_range_sliding* s, int64_t pane_index, const gf_points* pane, uint32_t* idx,
                           int64_t cap, int64_t* count, int32_t* closed, int64_t* window_end, int64_t* window_n);

/* Async window assembler for a batch in timestamp order (processing-time ingestion):
 * bounds (device int64[npanes + 1]) [j] = first i with ts[i] >= (first_pane + j) * pane_ms, so
 * pane first_pane + j is the slice [bounds[j], bounds[j+1]).  ts must be non-decreasing. */
int  gf_pane_bounds(gf_ctx* ctx, const int64_t* ts, int64_t n, int64_t pane_ms, int64_t first_pane, int32_t npanes,
                    int64_t* bounds);

/* ---- objID dictionaries ----------------------------------------------------------------
 * Device hash table + byte arena of the non-canonical objID Strings of a stream of windows.
 * gf_csv_parse uses the context's default dictionary (gf_ctx_objid_dict, owned by the
 * context); a JNI shim maps Point.objID Strings with gf_objid_intern and decodes result keys
 * (kNN objIDs) with gf_objid_decode.  Not thread-safe: one dictionary per calling thread. */
int  gf_objid_dict_create(gf_ctx* ctx, gf_objid_dict** out);
void gf_objid_dict_destroy(gf_objid_dict* d);
int  gf_ctx_objid_dict(gf_ctx* ctx, gf_objid_dict** out);
int  gf_objid_dict_size(const gf_objid_dict* d, int64_t* n);
/* Sync: keys of n host Strings, String i = bytes[offs[i], offs[i+1]) (offs: n+1 entries). */
int  gf_objid_intern(gf_objid_dict* d, const char* bytes, const int64_t* offs, int64_t n, int64_t* keys);
/* Sync: the Strings of n keys, String i = buf[offs[i], offs[i+1]) (offs: n+1 entries);
 * GF_ERR_CAPACITY when cap is too small (offs[n] = the bytes needed). */
int  gf_objid_decode(gf_objid_dict* d, const int64_t* keys, int64_t n, char* buf, int64_t cap, int64_t* offs);

/* ---- CSV / TSV ingest ----------------------------------------------------------------
 * Deserialization.CSVTSVToTSpatial(uGrid, dateFormat, delimiter, csvTsvSchemaAttr).map
 * (Deserialization.java:291-325) over a chunk of text lines, on the device.  Per line: '"'
 * removed, fields split on `delimiter` with the surrounding whitespace (split("\\s*" + delimiter
 * + "\\s*")), objID = the String field[objid_field] as its key (objID keys above; any String,
 * whitespace kept), ts = Long.valueOf(field[time_field]), x / y = Double.valueOf(...) correctly
 * rounded; with `grid`, the cell of Point(objID, x, y, ts, uGrid) (Point.java:98) as well.
 * Fields are read in the reference's order (objID, time, x, y): the first missing or
 * malformed one names the line's error. */
typedef struct {
  char delimiter;          /* ',' ';' '\t' ... (one character) */
  char reserved[3];
  int32_t objid_field;     /* csvTsvSchemaAttr.get(0) */
  int32_t time_field;      /* csvTsvSchemaAttr.get(1) */
  int32_t x_field;         /* csvTsvSchemaAttr.get(2) */
  int32_t y_field;         /* csvTsvSchemaAttr.get(3) */
} gf_csv_schema;
#define GF_CSV_OK              0
#define GF_CSV_NUMBER_FORMAT   1  /* Long.valueOf / Double.valueOf throw NumberFormatException */
#define GF_CSV_UNSUPPORTED     2  /* valid Java literal the device path does not take: hexadecimal, or
                                     > 19 significant digits within 1e-19 of a rounding boundary;
                                     or an objID field of 1 MiB or more */
#define GF_CSV_MISSING_FIELD   3  /* the reference's List.get throws IndexOutOfBoundsException */
#define GF_CSV_EMPTY_LINE      4  /* an empty line (a trailing newline at the end is fine) */
/* Sync.  text: device bytes [len], 16-byte aligned, complete lines separated by '\n' ("\r\n"
 * accepted; the last line may lack its '\n').  Outputs: device arrays of capacity cap (cx, cy
 * nullable, need grid).  *n_out = lines.  GF_ERR_CAPACITY if lines > cap (*n_out = lines);
 * GF_ERR_ARG on a bad line: *bad_line = its 0-based index, *bad_kind = GF_CSV_*. */
int gf_csv_parse(gf_ctx* ctx, const char* text, int64_t len, const gf_csv_schema* schema, const gf_grid* grid,
                 double* x, double* y, int64_t* objID, int64_t* ts, int32_t* cx, int32_t* cy, int64_t cap,
                 int64_t* n_out, int64_t* bad_line, int32_t* bad_kind);
/* As gf_csv_parse, objID keys from `dict` (NULL: the context's default dictionary). */
int gf_csv_parse_dict(gf_ctx* ctx, gf_objid_dict* dict, const char* text, int64_t len, const gf_csv_schema* schema,
                      const gf_grid* grid, double* x, double* y, int64_t* objID, int64_t* ts, int32_t* cx, int32_t* cy,
                      int64_t cap, int64_t* n_out, int64_t* bad_line, int32_t* bad_kind);

/* ---- GeoJSON ingest ------------------------------------------------------------------
 * Deserialization.GeoJSONToTSpatial(uGrid, dateFormat, propertyTimeStamp, propertyObjID).map
 * (Deserialization.java:149-211) over a chunk of lines, one JSON object per line: the ObjectNode
 * the map receives -- the Kafka record {"key":..,"value":..} (JSONKeyValueDeserializationSchema)
 * -- or, with value_lines = 1, the record's value itself (a Feature as
 * Serialization.PointToGeoJSONOutputSchema writes it).  Per line, in the map's order:
 *  - the record must be strict JSON as Jackson reads it (no NaN / Infinity, leading zeros,
 *    unescaped control bytes; UTF-8 checked structurally), else GF_CSV_MISSING_FIELD;
 *  - V = "value" (last duplicate wins, Jackson ObjectNode); missing / not an object:
 *    GF_CSV_MISSING_FIELD (the map's NullPointerException);
 *  - geometry = readGeoJSON(V) (jts-io-common 1.18.0 GeoJsonReader): V's "type" "Point" ->
 *    V's "coordinates"; on failure, and for "Feature" or a missing / non-string / unknown
 *    "type", the reference's catch branch readGeoJSON(V.geometry): "type" "Point" and
 *    "coordinates", else the line fails (GF_CSV_MISSING_FIELD; a non-number ordinate
 *    GF_CSV_NUMBER_FORMAT).  x, y = ordinates 0 and 1 (an integer literal is (double) of its
 *    long: "-0" -> 0.0);
 *  - from V's "properties" (absent or not an object: objID null, ts 0): ts from time_property
 *    -- date_format 0: Long.parseLong of the node's text (a JSON integer; anything else throws
 *    NumberFormatException: GF_CSV_NUMBER_FORMAT), date_format 1: the string value parsed as
 *    SimpleDateFormat("yyyy-MM-dd HH:mm:ss") (lenient field rollover) in a fixed UTC offset
 *    (tz_offset_minutes; DST not modelled), unparsable -> 0; objID from objid_property --
 *    node.toString() without '"': a string's content, an integer's digits ("-0" -> "0"),
 *    true / false / null as text; absent -> GF_OBJID_NULL.
 * GF_CSV_UNSUPPORTED (not restated, never guessed): geometry types other than Point (JTS builds
 * and validates them) and FeatureCollection; Point coordinates with fewer than two ordinates or
 * a non-number third; a number Jackson hands json-simple as text it cannot read back (a float
 * literal overflowing to Infinity, an integer literal outside long) anywhere on the line;
 * nesting deeper than 256; escapes in a taken string or in a member name of an object a value is
 * looked up in; non-integer or structured objID values; years before 1583 (Julian calendar). */
typedef struct {
  const char* objid_property;   /* propertyObjID (host C string, < 64 bytes); NULL: objID always null */
  const char* time_property;    /* propertyTimeStamp; NULL: ts always 0 */
  int32_t date_format;          /* 0: integer milliseconds; 1: "yyyy-MM-dd HH:mm:ss" */
  int32_t tz_offset_minutes;    /* date_format 1: offset of the reference JVM's default zone */
  int32_t value_lines;          /* 0: each line is the record {"key":..,"value":..}; 1: its value */
} gf_geojson_schema;
/* Same conventions as gf_csv_parse_dict (device text, outputs, capacity, first bad line). */
int gf_geojson_parse(gf_ctx* ctx, gf_objid_dict* dict, const char* text, int64_t len, const gf_geojson_schema* schema,
                     const gf_grid* grid, double* x, double* y, int64_t* objID, int64_t* ts, int32_t* cx,
                     int32_t* cy, int64_t cap, int64_t* n_out, int64_t* bad_line, int32_t* bad_kind);

/* ---- join (sync) --------------------------------------------------------------------
 * JoinQuery.getReplicatedPointQueryStream + PointPointJoinQuery.windowBased
 * (JoinQuery.java:73-90, PointPointJoinQuery.java:124-183).  pairs: device uint32[2*cap]
 * (ordinary idx, query idx), unordered.  *npairs = pairs found; GF_ERR_CAPACITY (with *npairs =
 * the exact count) if and only if that count > cap: the window's output regions are sized from
 * the context's previous join, and the pairs of a block that outgrows its region go to a device
 * spill sized so that every window whose pairs fit cap completes in one call. */
int gf_join_pp(gf_ctx* ctx, const gf_grid* ugrid, const gf_grid* qgrid, const gf_points* ordinary,
               const gf_points* query, double r, int approximate, int metric, uint32_t* pairs,
               int64_t cap, int64_t* npairs);
/* The same window join without a host wait: every launch stream-ordered on the context stream,
 * the pair count written by the last kernel to *total (device or mapped pinned memory), so the
 * next window's launches queue behind this one.  Pairs past cap are not written: the caller
 * re-runs the window with a larger buffer when *total > cap (*total = the exact count).  (r == 0
 * -- every cell a key --
 * takes the synchronous path and then stores *total.) */
int gf_join_pp_async(gf_ctx* ctx, const gf_grid* ugrid, const gf_grid* qgrid, const gf_points* ordinary,
                     const gf_points* query, double r, int approximate, int metric, uint32_t* pairs,
                     int64_t cap, unsigned long long* total);

/* Point-polygon window join: JoinQuery.getReplicatedPolygonQueryStream + PointPolygonJoinQuery
 * .windowBased (JoinQuery.java:93-115, PointPolygonJoinQuery.java:154-213).  Polygon q is
 * replicated to its own G_q u C_q keys (UniformGrid.java:193-206,399-411) on qgrid; point p
 * (key on ugrid, which must equal qgrid here) pairs with q if approximate or the JTS distance
 * (DistanceFunctions.java:33-36) is <= r.  The plan is the replicated polygon side (reusable
 * while the polygon set is unchanged); gf_range_plan_destroy frees it.  Run (sync): pairs =
 * device uint32[2*cap] (point idx, polygon idx), unordered; *npairs = pairs found,
 * GF_ERR_CAPACITY if > cap (pairs may be null with cap 0 to count). */
int gf_join_ppoly_plan_create(gf_ctx* ctx, const gf_grid* qgrid, const gf_polygons* polys, double r,
                              int approximate, int metric, gf_range_plan** out);
int gf_join_ppoly_run(gf_range_plan* plan, const gf_grid* ugrid, const gf_points* points, uint32_t* pairs,
                      int64_t cap, int64_t* npairs);
/* One-shot: plan create + run + destroy (a polygon stream's window). */
int gf_join_ppoly(gf_ctx* ctx, const gf_grid* ugrid, const gf_grid* qgrid, const gf_points* points,
                  const gf_polygons* polys, double r, int approximate, int metric, uint32_t* pairs,
                  int64_t cap, int64_t* npairs);

/* ---- pinned host memory ---------------------------------------------------------------
 * Mapped, portable host memory: kernels write kNN records straight into it (pass it as the
 * `result` of gf_knn_enqueue), so no copy kernel runs per window. */
int  gf_pinned_alloc(size_t bytes, void** ptr);
void gf_pinned_free(void* ptr);

/* ---- host windows -------------------------------------------------------------------- */
typedef struct gf_window gf_window;
/* Library-owned device SoA window (reused across windows: create once per plan / operator).
 * gf_window_upload copies on the window's own stream, after the work already enqueued on the
 * context (which may still read the old contents) and without blocking work enqueued later:
 * with two windows, upload(i+1) overlaps the evaluation of window i.  Pass NULL for columns
 * the query does not read (range / join: x, y = 16 B per point; kNN: x, y, objID; ts is never
 * read by window evaluation).  Host buffers from gf_pinned_alloc copy asynchronously at PCIe
 * rate; pageable ones are staged by the runtime.
 * gf_window_points MUST be called after each upload and before the evaluation that reads the
 * window: it orders the context's streams after the copy.  Columns not uploaded come back
 * NULL (a kNN plan then reports GF_ERR_ARG). */
int  gf_window_create(gf_ctx* ctx, int64_t capacity, gf_window** out);
void gf_window_destroy(gf_window* w);
int  gf_window_upload(gf_window* w, const double* x, const double* y, const int64_t* objID,
                      const int64_t* ts, int64_t n);
int  gf_window_points(gf_window* w, gf_points* out);
/* kNN windows at 16 B per point over PCIe (HipKnnWindowFunction.java:96-106 hands x, y, objID):
 * x and y are copied as gf_window_upload does, but the objID column stays in host memory --
 * objID_pinned must be gf_pinned_alloc memory -- and the kernels read it in place through the
 * mapping: only the few hundred candidates' objIDs ever cross the bus (the scan appends
 * (d, idx, objID) for points below the threshold; nothing else reads objID).  The column must
 * stay unchanged until the work that reads this window has completed. */
int  gf_window_upload_mapped(gf_window* w, const double* x, const double* y, const int64_t* objID_pinned, int64_t n);
/* *pinned = 1 when p lies in pinned host memory (gf_pinned_alloc / registered), so a shim can
 * take gf_window_upload_mapped for an objID column it was handed. */
int  gf_host_pinned(const void* p, int* pinned);

/* ---- synthetic input (host) ----------------------------------------------------------
 * java.util.Random(seed): x = minX + nextDouble()*(maxX-minX), then y likewise, per point
 * (cf. SyntheticGpsSource.java:23,40-41). */
int gf_synth_uniform(int64_t seed, int64_t n, double minX, double maxX, double minY, double maxY,
                     double* x, double* y);

#ifdef __cplusplus
}
#endif
#endif /* GEOFLINK_HIP_H */
