/*
 * geoflink_shim.h -- the plain-C core of the JNI shim (integration/jni/geoflink_jni.c): every
 * GeoFlinkHip native is a thin JNI wrapper (direct-buffer addresses and capacities, Java arrays,
 * exceptions) around one function here, which makes the whole gf_* call sequence of that entry
 * on host pointers.  No JNI types, so the core is compiled and exercised without a JDK:
 * tests/test_shim_native.py calls each function of libgeoflink_shim.so (ctypes) the way its JNI
 * wrapper does and compares the results with the oracle (built on the CPU suite, run on the GPU).
 *
 * Ownership: a shim_ctx is one Flink subtask's context (gf_ctx) plus the device buffers its
 * per-window calls reuse -- join windows, the ingest text buffer and columns, pinned result
 * staging -- so nothing is shared between contexts (two subtasks on two threads, or two contexts
 * of one subtask alternating windows).  Plans (kNN, range, sliding) hold their own device
 * windows.  Every function returns a GF_* status (include/geoflink_hip.h); on failure
 * shim_last_error(ctx) describes it.
 */
#ifndef GEOFLINK_SHIM_H
#define GEOFLINK_SHIM_H

#include <stdint.h>

#include "geoflink_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shim_ctx shim_ctx;
typedef struct shim_knn shim_knn;
typedef struct shim_range shim_range;
typedef struct shim_sliding shim_sliding;

int shim_ctx_create(int device, shim_ctx** out);
void shim_ctx_destroy(shim_ctx* c);
const char* shim_last_error(shim_ctx* c);
gf_ctx* shim_gf_ctx(shim_ctx* c);

/* ---- objID Strings <-> keys (the context's dictionary) ------------------------------------
 * Point.objID Strings of a window -> int64 keys (String i = bytes[offs[i], offs[i+1])), and
 * result keys -> Strings (GF_ERR_CAPACITY with offs[n] = bytes needed when cap is too small). */
int shim_objid_intern(shim_ctx* c, const char* bytes, const int64_t* offs, int64_t n, int64_t* keys);
int shim_objid_decode(shim_ctx* c, const int64_t* keys, int64_t n, char* buf, int64_t cap, int64_t* offs);

/* ---- kNN: PointPointKNNQuery.windowBased (PointPointKNNQuery.java:132-201) + windowAll merge
 * (KNNQuery.java:213-272), and PointPolygonKNNQuery (PointPolygonKNNQuery.java:245-317) ---- */
int shim_knn_plan(shim_ctx* c, const gf_grid* g, double qx, double qy, double r, int32_t k, shim_knn** out);
int shim_knn_polygon_plan(shim_ctx* c, const gf_grid* g, const gf_polygons* poly, double r, int32_t k,
                          int approximate, shim_knn** out);
void shim_knn_destroy(shim_knn* h);
/* one window (host x, y, objID keys) -> *m neighbours ascending (dist, objID); idx window-local */
/* pinned host memory for a window column the kernels read in place (objID: only the candidates'
 * keys cross PCIe -- gf_window_upload_mapped); upload() detects it with gf_host_pinned */
int shim_pinned_alloc(int64_t bytes, void** out);
void shim_pinned_free(void* p);
int shim_knn_window(shim_knn* h, const double* x, const double* y, const int64_t* objID, int64_t n, int64_t* out_objID,
                    double* out_dist, int64_t* out_idx, int32_t* m);
/* the plan's k: every kNN result array handed to the plan must hold at least this many entries */
int32_t shim_knn_k(const shim_knn* h);

/* ---- multi-GPU kNN: one subtask per GPU holds its cell-column band of every window; the
 * windowAll merge (PointPointKNNQuery.java:198-200, KNNQuery.java:213-272) becomes the RCCL
 * exchange of the C ABI (gf_knn_exchange_batch).  One process per GPU: rank 0's
 * shim_comm_unique_id (128 bytes) reaches every rank over the job's own channel (a Flink
 * broadcast), then shim_comm_create on each rank's context; one process: shim_comm_create_all. */
typedef struct shim_comm shim_comm;
int shim_comm_unique_id(uint8_t* id /* [GF_COMM_ID_BYTES] */);
int shim_comm_create(shim_ctx* c, const uint8_t* id, int32_t nranks, int32_t rank, shim_comm** out);
int shim_comm_create_all(int32_t ndev, const int* devices, shim_comm** out /* [ndev] */);
void shim_comm_destroy(shim_comm* comm);
/* this rank's band of one window (host x, y, objID keys; its points are global indices
 * index_base .. index_base + n - 1) -> the WHOLE window's *m neighbours, ascending (dist, objID),
 * identical on every rank.  Every rank calls it once per window, in the same order.  A rank whose
 * record needs the exact re-evaluation makes all ranks re-evaluate and exchange again. */
int shim_knn_window_sharded(shim_knn* h, shim_comm* comm, const double* x, const double* y, const int64_t* objID,
                            int64_t n, int64_t index_base, int64_t* out_objID, double* out_dist, int64_t* out_idx,
                            int32_t* m);
/* The batched, asynchronous form (the path bench.py --gpus N times): windows are ENQUEUED (this
 * rank's band uploaded into one of 2B device windows, its top-k record written on the device) and
 * every B-th enqueue issues ONE exchange of the last B windows' records -- by String
 * (gf_knn_exchange_strings_batch: the ranks' dictionaries differ, the windowAll merge dedupes by
 * Point.objID, KNNQuery.java:232-251) -- without a host wait; results are read per window after
 * its group's exchange.  Collective order: every rank makes the same begin / enqueue / flush /
 * result calls in the same order (result of a flagged window re-exchanges it on every rank).
 *   begin:   batch B (1..32), cap_bytes = the Strings of one record (e.g. 32 k)
 *   enqueue: *ticket = the window's sequence number; GF_ERR_ARG when the window 2B tickets back
 *            (same slot) was not read yet
 *   flush:   exchange the enqueued windows of an incomplete group now (end of stream, a timer)
 *   result:  a ticket whose group was exchanged -> *m entries, ascending (dist, String): dist,
 *            global idx (index_base + window position); `owned` marks the entries of this rank's
 *            band (index_base <= idx < index_base + n), so each rank emits its own Points.
 *            GF_ERR_ARG for a ticket not exchanged (call flush) or already read. */
int shim_knn_sharded_begin(shim_knn* h, shim_comm* comm, int32_t batch, int64_t cap_bytes);
int shim_knn_sharded_enqueue(shim_knn* h, const double* x, const double* y, const int64_t* objID, int64_t n,
                             int64_t index_base, int64_t* ticket);
int shim_knn_sharded_flush(shim_knn* h);
int shim_knn_sharded_result(shim_knn* h, int64_t ticket, double* out_dist, int64_t* out_idx, int32_t* owned,
                            int32_t* m);

/* ---- sliding kNN: SlidingProcessingTimeWindows.of(size, slide) around the kNN apply
 * (PointPointKNNQuery.java:158,198-200) -- the pane engine (gf_knn_sliding_*) ---------------- */
int shim_sliding_create(shim_knn* plan, int64_t size_ms, int64_t slide_ms, shim_sliding** out);
void shim_sliding_destroy(shim_sliding* s);
int shim_sliding_pane_ms(const shim_sliding* s, int64_t* pane_ms);
/* push pane `pane_index` (host columns, n may be 0); *closed = 1 when a window closed with it,
 * *window_end its end -- then decode it with shim_sliding_decode (a pending window's record is
 * completed by the next push or by shim_sliding_flush) */
int shim_sliding_push(shim_sliding* s, int64_t pane_index, const double* x, const double* y, const int64_t* objID,
                      int64_t n, int32_t* closed, int64_t* window_end);
int shim_sliding_flush(shim_sliding* s);
shim_knn* shim_sliding_plan(shim_sliding* s);  /* the kNN plan the engine runs (its k sizes decode's arrays) */
int shim_sliding_decode(shim_sliding* s, int64_t window_end, int64_t* out_objID, double* out_dist, int64_t* out_idx,
                        int32_t* m);

/* ---- range: PointPointRangeQuery / PointPolygonRangeQuery window apply
 * (PointPointRangeQuery.java:150-186, PointPolygonRangeQuery.java:170-204) ------------------- */
int shim_range_plan(shim_ctx* c, const gf_grid* g, const double* qx, const double* qy, int32_t nq, double r,
                    int approximate, shim_range** out);
int shim_range_polygon_plan(shim_ctx* c, const gf_grid* g, const gf_polygons* polys, double r, int approximate,
                            shim_range** out);
void shim_range_destroy(shim_range* h);
/* emitted point indices, ascending, into out_idx[cap]; *count = all of them (GF_ERR_CAPACITY if
 * > cap).  One device pass: bitmap, then the index list into pinned memory, one stream sync. */
int shim_range_window(shim_range* h, const double* x, const double* y, int64_t n, int32_t* out_idx, int64_t cap,
                      int64_t* count);
/* approximate point-point range with |Q| > 1: the reference's apply emits a candidate-cell point
 * once per query point (PointPointRangeQuery.java:158-161), so those points of the LAST window
 * (ascending, a subset of shim_range_window's list) are listed here -- emit each |Q| times in
 * all.  *count = 0 for every other plan. */
int shim_range_window_multi(shim_range* h, int32_t* out_idx, int64_t cap, int64_t* count);

/* ---- sliding range: SlidingProcessingTimeWindows.of(size, slide) around the range apply
 * (PointPointRangeQuery.java:149-186) -- the pane engine (gf_range_sliding_*) ------------------ */
typedef struct shim_range_sliding shim_range_sliding;
int shim_range_sliding_create(shim_range* plan, int64_t size_ms, int64_t slide_ms, shim_range_sliding** out);
void shim_range_sliding_destroy(shim_range_sliding* s);
int shim_range_sliding_pane_ms(const shim_range_sliding* s, int64_t* pane_ms);
/* push pane `pane_index` (host x, y; n may be 0).  When it closes a window holding a point:
 * *window_end = its end, *idx = the window's emitted points (positions in the window's panes
 * concatenated, ascending; in the shim's pinned staging until the next push), *count; else
 * *window_end = -1. */
int shim_range_sliding_push(shim_range_sliding* s, int64_t pane_index, const double* x, const double* y, int64_t n,
                            int64_t* window_end, const uint32_t** idx, int64_t* count);

/* ---- joins (JoinQuery.java:73-115, PointPointJoinQuery.java:148-182,
 * PointPolygonJoinQuery.java:154-213): pairs (ordinary / point index, query / polygon index) ---
 * The pairs stay in the context's pinned staging until the next join on it: *pairs points there
 * (2 * *m uint32). */
int shim_join_window(shim_ctx* c, const gf_grid* ug, const gf_grid* qg, const double* ox, const double* oy, int64_t no,
                     const double* qx, const double* qy, int64_t nq, double r, int approximate, const uint32_t** pairs,
                     int64_t* m);
int shim_polygon_join_window(shim_ctx* c, const gf_grid* g, const double* x, const double* y, int64_t n,
                             const gf_polygons* polys, double r, int approximate, const uint32_t** pairs, int64_t* m);

/* ---- ingest (Deserialization.java:149-211, 291-325): a chunk of complete lines -> host columns
 * of capacity cap (x, y, objID keys, ts); *n = lines.  Bad line: GF_ERR_ARG with *bad_line,
 * *bad_kind (GF_CSV_*). ---------------------------------------------------------------------- */
int shim_csv_parse(shim_ctx* c, const char* text, int64_t len, const gf_csv_schema* schema, double* x, double* y,
                   int64_t* objID, int64_t* ts, int64_t cap, int64_t* n, int64_t* bad_line, int32_t* bad_kind);
int shim_geojson_parse(shim_ctx* c, const char* text, int64_t len, const gf_geojson_schema* schema, double* x,
                       double* y, int64_t* objID, int64_t* ts, int64_t cap, int64_t* n, int64_t* bad_line,
                       int32_t* bad_kind);

#ifdef __cplusplus
}
#endif
#endif
