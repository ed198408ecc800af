/*
 * geoflink_jni.c -- the C side of the JNI shim behind GeoFlink.native_.GeoFlinkHip (see
 * INTEGRATION.md).  NOT COMPILED in this repository: the build image has no JDK, so jni.h is
 * absent.  It is kept as a real source file; on a machine with a JDK:
 *
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ integration/jni/geoflink_jni.c \
 *       -Lspatialflink_amd -lgeoflink_hip -L/opt/rocm/lib -lamdhip64 -o libgeoflink_jni.so
 *
 * Ownership: a plan handle is a shim struct holding the library plan, its context and the
 * device window(s) it uploads into -- created once per continuous query and reused window
 * after window (gf_window_upload into the same device buffers; only the columns the query
 * reads are copied: x, y for range / join, + objID for kNN).  Errors become Java exceptions
 * (IllegalArgumentException for GF_ERR_ARG, RuntimeException otherwise: the reference's
 * System.exit(1) on non-positive candidate layers is GF_ERR_LAYERS).
 */
#include <jni.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "geoflink_hip.h"

static void throw_status(JNIEnv* env, int st, gf_ctx* ctx) {
  const char* cls = st == GF_ERR_ARG ? "java/lang/IllegalArgumentException" : "java/lang/RuntimeException";
  (*env)->ThrowNew(env, (*env)->FindClass(env, cls), ctx ? gf_ctx_last_error(ctx) : gf_status_string(st));
}

static void* buf(JNIEnv* env, jobject b) { return b ? (*env)->GetDirectBufferAddress(env, b) : NULL; }

/* a device window of at least n points, grown (recreated) only when a window is larger */
typedef struct {
  gf_window* w;
  int64_t cap;
} cached_window;

static int window_for(gf_ctx* ctx, cached_window* c, int64_t n) {
  if (c->w && c->cap >= n) return GF_OK;
  if (c->w) gf_window_destroy(c->w);
  c->w = NULL;
  c->cap = n > 1024 ? n + n / 4 : 1024;
  return gf_window_create(ctx, c->cap, &c->w);
}

/* upload the given columns and return the device points (ordered after the copy) */
static int upload(gf_ctx* ctx, cached_window* c, const double* x, const double* y, const int64_t* objID, int64_t n,
                  gf_points* pts) {
  int st = window_for(ctx, c, n);
  if (!st) st = gf_window_upload(c->w, x, y, objID, NULL, n);
  if (!st) st = gf_window_points(c->w, pts);
  return st;
}

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_ctxCreate(JNIEnv* env, jclass cls, jint dev) {
  gf_ctx* ctx = NULL;
  int st = gf_ctx_create(dev, &ctx);
  if (st) throw_status(env, st, NULL);
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_ctxDestroy(JNIEnv* env, jclass cls, jlong ctx) {
  gf_ctx_destroy((gf_ctx*)(intptr_t)ctx);
}

/* ---- kNN ------------------------------------------------------------------------------ */
typedef struct {
  gf_ctx* ctx;
  gf_knn_plan* plan;
  cached_window win;
} knn_handle;

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnPlan(JNIEnv* env, jclass cls, jlong ctxh, jint n,
    jdouble minX, jdouble maxX, jdouble minY, jdouble maxY, jdouble qx, jdouble qy, jdouble r, jint k) {
  gf_ctx* ctx = (gf_ctx*)(intptr_t)ctxh;
  knn_handle* h = (knn_handle*)calloc(1, sizeof(knn_handle));
  gf_grid g;
  int st = h ? gf_grid_make(n, minX, maxX, minY, maxY, &g) : GF_ERR_NOMEM;
  if (!st) st = gf_knn_pp_plan_create(ctx, &g, qx, qy, r, k, GF_METRIC_SQRT, &h->plan);
  if (st) {
    free(h);
    throw_status(env, st, ctx);
    return 0;
  }
  h->ctx = ctx;
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnPlanDestroy(JNIEnv* env, jclass cls, jlong p) {
  knn_handle* h = (knn_handle*)(intptr_t)p;
  if (!h) return;
  if (h->win.w) gf_window_destroy(h->win.w);
  gf_knn_plan_destroy(h->plan);
  free(h);
}

/* PointPointKNNQuery.windowBased apply + windowAll merge for one window */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnWindow(JNIEnv* env, jclass cls, jlong p, jobject bx,
    jobject by, jobject bo, jint n, jlongArray oo, jdoubleArray od, jlongArray oi) {
  knn_handle* h = (knn_handle*)(intptr_t)p;
  gf_points pts;
  int32_t m = 0;
  int st = upload(h->ctx, &h->win, buf(env, bx), buf(env, by), buf(env, bo), n, &pts);
  jlong* po = (*env)->GetPrimitiveArrayCritical(env, oo, NULL);
  jdouble* pd = (*env)->GetPrimitiveArrayCritical(env, od, NULL);
  jlong* pi = (*env)->GetPrimitiveArrayCritical(env, oi, NULL);
  if (!st) st = gf_knn_run(h->plan, &pts, (int64_t*)po, pd, (int64_t*)pi, &m);
  (*env)->ReleasePrimitiveArrayCritical(env, oi, pi, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, od, pd, 0);
  (*env)->ReleasePrimitiveArrayCritical(env, oo, po, 0);
  if (st) {
    throw_status(env, st, h->ctx);
    return 0;
  }
  return m;
}

/* ---- range ---------------------------------------------------------------------------- */
typedef struct {
  gf_ctx* ctx;
  gf_range_plan* plan;
  cached_window win;
  uint64_t* bitmap;   /* device */
  uint32_t* idx;      /* device */
  int64_t cap;
} range_handle;

static jlong range_handle_new(JNIEnv* env, gf_ctx* ctx, gf_range_plan* plan, int st) {
  range_handle* h = st ? NULL : (range_handle*)calloc(1, sizeof(range_handle));
  if (st || !h) {
    if (plan) gf_range_plan_destroy(plan);
    throw_status(env, st ? st : GF_ERR_NOMEM, ctx);
    return 0;
  }
  h->ctx = ctx;
  h->plan = plan;
  return (jlong)(intptr_t)h;
}

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangePlan(JNIEnv* env, jclass cls, jlong ctxh, jint n,
    jdouble minX, jdouble maxX, jdouble minY, jdouble maxY, jdoubleArray jqx, jdoubleArray jqy, jdouble r,
    jboolean approximate) {
  gf_ctx* ctx = (gf_ctx*)(intptr_t)ctxh;
  gf_grid g;
  gf_range_plan* plan = NULL;
  int st = gf_grid_make(n, minX, maxX, minY, maxY, &g);
  jdouble* qx = (*env)->GetDoubleArrayElements(env, jqx, NULL);
  jdouble* qy = (*env)->GetDoubleArrayElements(env, jqy, NULL);
  if (!st) st = gf_range_pp_plan_create(ctx, &g, qx, qy, (*env)->GetArrayLength(env, jqx), r, approximate,
                                        GF_METRIC_SQRT, &plan);
  (*env)->ReleaseDoubleArrayElements(env, jqy, qy, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, jqx, qx, JNI_ABORT);
  return range_handle_new(env, ctx, plan, st);
}

static void polygons_get(JNIEnv* env, jintArray jro, jintArray jvo, jdoubleArray jvx, jdoubleArray jvy, gf_polygons* P) {
  P->npoly = (*env)->GetArrayLength(env, jro) - 1;
  P->ring_off = (*env)->GetIntArrayElements(env, jro, NULL);
  P->vert_off = (*env)->GetIntArrayElements(env, jvo, NULL);
  P->vx = (*env)->GetDoubleArrayElements(env, jvx, NULL);
  P->vy = (*env)->GetDoubleArrayElements(env, jvy, NULL);
}

static void polygons_release(JNIEnv* env, jintArray jro, jintArray jvo, jdoubleArray jvx, jdoubleArray jvy,
                             gf_polygons* P) {
  (*env)->ReleaseDoubleArrayElements(env, jvy, (jdouble*)P->vy, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, jvx, (jdouble*)P->vx, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, jvo, (jint*)P->vert_off, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, jro, (jint*)P->ring_off, JNI_ABORT);
}

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangePolygonPlan(JNIEnv* env, jclass cls, jlong ctxh,
    jint n, jdouble minX, jdouble maxX, jdouble minY, jdouble maxY, jintArray jro, jintArray jvo, jdoubleArray jvx,
    jdoubleArray jvy, jdouble r, jboolean approximate) {
  gf_ctx* ctx = (gf_ctx*)(intptr_t)ctxh;
  gf_grid g;
  gf_polygons P;
  gf_range_plan* plan = NULL;
  int st = gf_grid_make(n, minX, maxX, minY, maxY, &g);
  polygons_get(env, jro, jvo, jvx, jvy, &P);
  if (!st) st = gf_range_ppoly_plan_create(ctx, &g, &P, r, approximate, GF_METRIC_SQRT, &plan);
  polygons_release(env, jro, jvo, jvx, jvy, &P);
  return range_handle_new(env, ctx, plan, st);
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangePlanDestroy(JNIEnv* env, jclass cls, jlong p) {
  range_handle* h = (range_handle*)(intptr_t)p;
  if (!h) return;
  if (h->win.w) gf_window_destroy(h->win.w);
  hipFree(h->bitmap);
  hipFree(h->idx);
  gf_range_plan_destroy(h->plan);
  free(h);
}

/* PointPointRangeQuery / PointPolygonRangeQuery window apply: emitted indices, ascending */
JNIEXPORT jintArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeWindow(JNIEnv* env, jclass cls, jlong p,
    jobject bx, jobject by, jint n) {
  range_handle* h = (range_handle*)(intptr_t)p;
  gf_points pts;
  int64_t count = 0;
  int st = upload(h->ctx, &h->win, buf(env, bx), buf(env, by), NULL, n, &pts);
  if (!st && h->cap < n) {  /* per-plan result buffers, grown with the window */
    hipFree(h->bitmap);
    hipFree(h->idx);
    h->bitmap = NULL;
    h->idx = NULL;
    h->cap = h->win.cap;
    if (hipMalloc((void**)&h->bitmap, 8 * (size_t)((h->cap + 63) / 64)) != hipSuccess ||
        hipMalloc((void**)&h->idx, 4 * (size_t)h->cap) != hipSuccess) {
      h->cap = 0;
      st = GF_ERR_NOMEM;
    }
  }
  if (!st) st = gf_range_run(h->plan, &pts, h->bitmap, NULL, NULL);
  if (!st) st = gf_bitmap_to_indices(h->ctx, h->bitmap, n, h->idx, h->cap, &count);
  jintArray out = NULL;
  if (!st) {
    out = (*env)->NewIntArray(env, (jsize)count);
    jint* po = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    if (hipMemcpy(po, h->idx, 4 * (size_t)count, hipMemcpyDeviceToHost) != hipSuccess) st = GF_ERR_HIP;
    (*env)->ReleasePrimitiveArrayCritical(env, out, po, 0);
  }
  if (st) throw_status(env, st, h->ctx);
  return out;
}

/* ---- joins ---------------------------------------------------------------------------- */
static int grid_of(JNIEnv* env, jdoubleArray jg, gf_grid* g) {
  jdouble* d = (*env)->GetDoubleArrayElements(env, jg, NULL);  /* n, minX, maxX, minY, maxY */
  int st = gf_grid_make((int32_t)d[0], d[1], d[2], d[3], d[4], g);
  (*env)->ReleaseDoubleArrayElements(env, jg, d, JNI_ABORT);
  return st;
}

/* device pairs -> a Java long[2m] of (ordinary / point index, query / polygon index) */
static jlongArray pairs_out(JNIEnv* env, const uint32_t* dev_pairs, int64_t m, int* st) {
  uint32_t* host = (uint32_t*)malloc(8 * (size_t)(m > 0 ? m : 1));
  jlongArray out = NULL;
  if (!host || hipMemcpy(host, dev_pairs, 8 * (size_t)m, hipMemcpyDeviceToHost) != hipSuccess) {
    *st = GF_ERR_HIP;
  } else {
    out = (*env)->NewLongArray(env, (jsize)(2 * m));
    jlong* po = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
    for (int64_t i = 0; i < 2 * m; ++i) po[i] = host[i];
    (*env)->ReleasePrimitiveArrayCritical(env, out, po, 0);
  }
  free(host);
  return out;
}

/* JoinQuery.getReplicatedPointQueryStream + PointPointJoinQuery.windowBased for one window pair.
 * Two-phase capacity: count with pairs = NULL, then allocate and run. */
JNIEXPORT jlongArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_joinWindow(JNIEnv* env, jclass cls, jlong ctxh,
    jdoubleArray jug, jdoubleArray jqg, jobject box, jobject boy, jint no, jobject bqx, jobject bqy, jint nq,
    jdouble r, jboolean approximate) {
  gf_ctx* ctx = (gf_ctx*)(intptr_t)ctxh;
  static __thread cached_window wo, wq;  /* one context per subtask thread */
  gf_grid ug, qg;
  gf_points po, pq;
  int64_t m = 0;
  uint32_t* dev_pairs = NULL;
  int st = grid_of(env, jug, &ug);
  if (!st) st = grid_of(env, jqg, &qg);
  if (!st) st = upload(ctx, &wo, buf(env, box), buf(env, boy), NULL, no, &po);
  if (!st) st = upload(ctx, &wq, buf(env, bqx), buf(env, bqy), NULL, nq, &pq);
  if (!st) st = gf_join_pp(ctx, &ug, &qg, &po, &pq, r, approximate, GF_METRIC_SQRT, NULL, 0, &m);
  if (st == GF_ERR_CAPACITY) {
    st = hipMalloc((void**)&dev_pairs, 8 * (size_t)(m > 0 ? m : 1)) == hipSuccess ? GF_OK : GF_ERR_NOMEM;
    if (!st) st = gf_join_pp(ctx, &ug, &qg, &po, &pq, r, approximate, GF_METRIC_SQRT, dev_pairs, m, &m);
  }
  jlongArray out = NULL;
  if (!st) out = pairs_out(env, dev_pairs, m, &st);
  hipFree(dev_pairs);
  if (st) throw_status(env, st, ctx);
  return out;
}

/* JoinQuery.getReplicatedPolygonQueryStream + PointPolygonJoinQuery.windowBased */
JNIEXPORT jlongArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_polygonJoinWindow(JNIEnv* env, jclass cls,
    jlong ctxh, jdoubleArray jg, jobject bx, jobject by, jint n, jintArray jro, jintArray jvo, jdoubleArray jvx,
    jdoubleArray jvy, jdouble r, jboolean approximate) {
  gf_ctx* ctx = (gf_ctx*)(intptr_t)ctxh;
  static __thread cached_window wp;
  gf_grid g;
  gf_polygons P;
  gf_points pts;
  gf_range_plan* plan = NULL;
  int64_t m = 0;
  uint32_t* dev_pairs = NULL;
  int st = grid_of(env, jg, &g);
  polygons_get(env, jro, jvo, jvx, jvy, &P);
  if (!st) st = gf_join_ppoly_plan_create(ctx, &g, &P, r, approximate, GF_METRIC_SQRT, &plan);
  polygons_release(env, jro, jvo, jvx, jvy, &P);
  if (!st) st = upload(ctx, &wp, buf(env, bx), buf(env, by), NULL, n, &pts);
  if (!st) st = gf_join_ppoly_run(plan, &g, &pts, NULL, 0, &m);
  if (st == GF_ERR_CAPACITY) {
    st = hipMalloc((void**)&dev_pairs, 8 * (size_t)(m > 0 ? m : 1)) == hipSuccess ? GF_OK : GF_ERR_NOMEM;
    if (!st) st = gf_join_ppoly_run(plan, &g, &pts, dev_pairs, m, &m);
  }
  jlongArray out = NULL;
  if (!st) out = pairs_out(env, dev_pairs, m, &st);
  hipFree(dev_pairs);
  if (plan) gf_range_plan_destroy(plan);
  if (st) throw_status(env, st, ctx);
  return out;
}

/* ---- ingest --------------------------------------------------------------------------- */
/* device text buffer, per subtask thread, grown on demand */
static int device_text(JNIEnv* env, jobject btext, jint len, char** dev) {
  static __thread char* d = NULL;
  static __thread size_t cap = 0;
  if ((size_t)len > cap) {
    hipFree(d);
    d = NULL;
    cap = (size_t)len + (size_t)len / 4 + 4096;
    if (hipMalloc((void**)&d, cap) != hipSuccess) {
      cap = 0;
      return GF_ERR_NOMEM;
    }
  }
  if (len && hipMemcpy(d, buf(env, btext), (size_t)len, hipMemcpyHostToDevice) != hipSuccess) return GF_ERR_HIP;
  *dev = d;
  return GF_OK;
}

/* parsed device columns -> the caller's direct buffers */
static int columns_out(JNIEnv* env, int64_t n, double* x, double* y, int64_t* o, int64_t* t, jobject bx, jobject by,
                       jobject bo, jobject bt) {
  const size_t b = 8 * (size_t)n;
  if (hipMemcpy(buf(env, bx), x, b, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(buf(env, by), y, b, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(buf(env, bo), o, b, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(buf(env, bt), t, b, hipMemcpyDeviceToHost) != hipSuccess)
    return GF_ERR_HIP;
  return GF_OK;
}

static jint parse_common(JNIEnv* env, gf_ctx* ctx, jobject btext, jint len, jobject bx, jobject by, jobject bo,
                         jobject bt, jint capacity, int geojson, const void* schema) {
  char* text = NULL;
  double *x = NULL, *y = NULL;
  int64_t *o = NULL, *t = NULL, n = 0, bad_line = -1;
  int32_t bad_kind = 0;
  const size_t b = 8 * (size_t)(capacity > 0 ? capacity : 1);
  int st = device_text(env, btext, len, &text);
  if (!st && (hipMalloc((void**)&x, b) != hipSuccess || hipMalloc((void**)&y, b) != hipSuccess ||
              hipMalloc((void**)&o, b) != hipSuccess || hipMalloc((void**)&t, b) != hipSuccess))
    st = GF_ERR_NOMEM;
  if (!st)
    st = geojson ? gf_geojson_parse(ctx, NULL, text, len, (const gf_geojson_schema*)schema, NULL, x, y, o, t, NULL,
                                    NULL, capacity, &n, &bad_line, &bad_kind)
                 : gf_csv_parse(ctx, text, len, (const gf_csv_schema*)schema, NULL, x, y, o, t, NULL, NULL, capacity,
                                &n, &bad_line, &bad_kind);
  if (!st) st = columns_out(env, n, x, y, o, t, bx, by, bo, bt);
  hipFree(x);
  hipFree(y);
  hipFree(o);
  hipFree(t);
  if (st) {
    throw_status(env, st, ctx);  /* GF_ERR_ARG: the reference's map would have thrown on bad_line */
    return 0;
  }
  return (jint)n;
}

/* Deserialization.CSVTSVToTSpatial.map over a chunk of complete lines */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_csvParse(JNIEnv* env, jclass cls, jlong ctxh, jobject btext,
    jint len, jchar delimiter, jintArray jschema, jobject bx, jobject by, jobject bo, jobject bt, jint capacity) {
  gf_csv_schema sc;
  memset(&sc, 0, sizeof sc);
  jint* s = (*env)->GetIntArrayElements(env, jschema, NULL);
  sc.delimiter = (char)delimiter;
  sc.objid_field = s[0];
  sc.time_field = s[1];
  sc.x_field = s[2];
  sc.y_field = s[3];
  (*env)->ReleaseIntArrayElements(env, jschema, s, JNI_ABORT);
  return parse_common(env, (gf_ctx*)(intptr_t)ctxh, btext, len, bx, by, bo, bt, capacity, 0, &sc);
}

/* Deserialization.GeoJSONToTSpatial.map over a chunk of lines (oID / timestamp properties, the
 * reference's Serialization names; date strings "yyyy-MM-dd HH:mm:ss" in the JVM's zone) */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_geoJsonParse(JNIEnv* env, jclass cls, jlong ctxh,
    jobject btext, jint len, jobject bx, jobject by, jobject bo, jobject bt, jint capacity) {
  gf_geojson_schema sc;
  sc.objid_property = "oID";
  sc.time_property = "timestamp";
  sc.date_format = 1;
  sc.tz_offset_minutes = 0;  /* the shim sets TimeZone.getDefault().getRawOffset() / 60000 here */
  return parse_common(env, (gf_ctx*)(intptr_t)ctxh, btext, len, bx, by, bo, bt, capacity, 1, &sc);
}
