/*
 * geoflink_jni.c -- the JNI side of the shim behind GeoFlink.native_.GeoFlinkHip (see
 * INTEGRATION.md).  Every native is a thin wrapper: it checks the Java arguments (direct-buffer
 * capacities, array lengths), pins them, and calls ONE function of the plain-C core
 * (geoflink_shim.h), which makes the whole gf_* call sequence.  The core is compiled and run
 * without a JDK as libgeoflink_shim.so, driven by tests/test_shim_native.py; this file needs jni.h,
 * which the build image lacks, so it is built on a machine with a JDK:
 *
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ integration/jni/geoflink_jni.c \
 *       integration/jni/geoflink_shim.c -Lspatialflink_amd -lgeoflink_hip \
 *       -L/opt/rocm/lib -lamdhip64 -o libgeoflink_jni.so
 *
 * Handles are native pointers in a long: a context (shim_ctx: one Flink subtask's gf_ctx plus
 * the device buffers its windows reuse), and plans (kNN, range, sliding kNN) that hold their
 * own device windows.  Nothing is shared between contexts.  Errors become Java exceptions:
 * IllegalArgumentException for GF_ERR_ARG (the reference's map / apply would have thrown), an
 * IndexOutOfBoundsException for a buffer smaller than the call needs, RuntimeException otherwise
 * (the reference's System.exit(1) on non-positive candidate layers is GF_ERR_LAYERS).
 */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "geoflink_shim.h"

#define CTX(h) ((shim_ctx*)(intptr_t)(h))

static void throw_msg(JNIEnv* env, const char* cls, const char* msg) {
  if ((*env)->ExceptionCheck(env)) return;
  (*env)->ThrowNew(env, (*env)->FindClass(env, cls), msg);
}
static int throw_status(JNIEnv* env, int st, shim_ctx* c) {
  if (st)
    throw_msg(env, st == GF_ERR_ARG ? "java/lang/IllegalArgumentException" : "java/lang/RuntimeException",
              c ? shim_last_error(c) : gf_status_string(st));
  return st;
}

/* a direct ByteBuffer holding at least `bytes` -> its address; NULL + IndexOutOfBounds otherwise */
static void* direct(JNIEnv* env, jobject b, int64_t bytes, const char* what) {
  if ((*env)->ExceptionCheck(env)) return NULL;  /* an earlier argument already threw */
  if (bytes <= 0) return b ? (*env)->GetDirectBufferAddress(env, b) : NULL;
  void* p = b ? (*env)->GetDirectBufferAddress(env, b) : NULL;
  if (!p) {
    throw_msg(env, "java/lang/IllegalArgumentException", what);
    return NULL;
  }
  if ((*env)->GetDirectBufferCapacity(env, b) < bytes) {
    throw_msg(env, "java/lang/IndexOutOfBoundsException", what);
    return NULL;
  }
  return p;
}
static int need_len(JNIEnv* env, jarray a, jsize n, const char* what) {
  if (!a || (*env)->GetArrayLength(env, a) < n) {
    throw_msg(env, "java/lang/IndexOutOfBoundsException", what);
    return 0;
  }
  return 1;
}

/* the three result arrays of a kNN call hold at least the PLAN's k entries (the shim writes up to
 * that many, whatever k the Java caller passes) */
static int need_knn_out(JNIEnv* env, const shim_knn* h, jarray oo, jarray od, jarray oi, const char* what) {
  const jsize k = (jsize)shim_knn_k(h);
  return need_len(env, oo, k, what) && need_len(env, od, k, what) && need_len(env, oi, k, what);
}
/* Get<Type>ArrayElements can fail (out of memory): NULL throws, release what was pinned */
static int pinned_ok(JNIEnv* env, const void* a, const void* b, const void* c) {
  if (a && b && c) return 1;
  throw_msg(env, "java/lang/OutOfMemoryError", "pinning result arrays");
  return 0;
}

/* UniformGrid(n, minX, maxX, minY, maxY) as double[5] */
static int grid_of(JNIEnv* env, jdoubleArray jg, gf_grid* g) {
  if (!need_len(env, jg, 5, "grid: {n, minX, maxX, minY, maxY}")) return GF_ERR_ARG;
  jdouble d[5];
  (*env)->GetDoubleArrayRegion(env, jg, 0, 5, d);
  int st = gf_grid_make((int32_t)d[0], d[1], d[2], d[3], d[4], g);
  if (st) throw_msg(env, "java/lang/IllegalArgumentException", "grid");
  return st;
}

/* polygons as CSR int[] ringOff (npoly+1), int[] vertOff (nrings+1), double[] vx, vy */
typedef struct {
  jintArray ro, vo;
  jdoubleArray vx, vy;
  gf_polygons P;
} jpolys;
static int polys_get(JNIEnv* env, jpolys* j) {
  memset(&j->P, 0, sizeof j->P);
  if (!j->ro || !j->vo || !j->vx || !j->vy) {
    throw_msg(env, "java/lang/IllegalArgumentException", "polygons");
    return GF_ERR_ARG;
  }
  const jsize npoly = (*env)->GetArrayLength(env, j->ro) - 1;
  const jsize nv = (*env)->GetArrayLength(env, j->vx);
  if (npoly < 0 || (*env)->GetArrayLength(env, j->vy) != nv) {
    throw_msg(env, "java/lang/IllegalArgumentException", "polygons: ringOff / vx / vy");
    return GF_ERR_ARG;
  }
  j->P.npoly = npoly;
  j->P.ring_off = (*env)->GetIntArrayElements(env, j->ro, NULL);
  j->P.vert_off = (*env)->GetIntArrayElements(env, j->vo, NULL);
  j->P.vx = (*env)->GetDoubleArrayElements(env, j->vx, NULL);
  j->P.vy = (*env)->GetDoubleArrayElements(env, j->vy, NULL);
  return GF_OK;  /* offsets are validated by the library (GF_ERR_ARG) */
}
static void polys_release(JNIEnv* env, jpolys* j) {
  if (j->P.vy) (*env)->ReleaseDoubleArrayElements(env, j->vy, (jdouble*)j->P.vy, JNI_ABORT);
  if (j->P.vx) (*env)->ReleaseDoubleArrayElements(env, j->vx, (jdouble*)j->P.vx, JNI_ABORT);
  if (j->P.vert_off) (*env)->ReleaseIntArrayElements(env, j->vo, (jint*)j->P.vert_off, JNI_ABORT);
  if (j->P.ring_off) (*env)->ReleaseIntArrayElements(env, j->ro, (jint*)j->P.ring_off, JNI_ABORT);
}

/* ---- context ---------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_ctxCreate(JNIEnv* env, jclass cls, jint dev) {
  shim_ctx* c = NULL;
  throw_status(env, shim_ctx_create(dev, &c), NULL);
  return (jlong)(intptr_t)c;
}
JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_ctxDestroy(JNIEnv* env, jclass cls, jlong ctx) {
  shim_ctx_destroy(CTX(ctx));
}

/* ---- objID Strings <-> keys --------------------------------------------------------------
 * Java encodes the window's objID Strings as UTF-8 into one byte[] with long[] offsets (n + 1);
 * decode returns the bytes and fills offsets, Java builds new String(bytes, off, len, UTF_8)
 * (not NewStringUTF: modified UTF-8 differs for NUL and supplementary characters). */
JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_objidIntern(JNIEnv* env, jclass cls, jlong ctx,
    jbyteArray jbytes, jlongArray joffs, jint n, jlongArray jkeys) {
  if (n < 0 || !need_len(env, joffs, n + 1, "objidIntern: offs") || !need_len(env, jkeys, n, "objidIntern: keys"))
    return;
  jlong* offs = (*env)->GetLongArrayElements(env, joffs, NULL);
  const jlong total = offs[n];
  if (offs[0] != 0 || total < 0 || !need_len(env, jbytes, (jsize)total, "objidIntern: bytes")) {
    (*env)->ReleaseLongArrayElements(env, joffs, offs, JNI_ABORT);
    throw_msg(env, "java/lang/IllegalArgumentException", "objidIntern: offs");
    return;
  }
  jbyte* bytes = (*env)->GetByteArrayElements(env, jbytes, NULL);
  jlong* keys = (*env)->GetLongArrayElements(env, jkeys, NULL);
  int st = shim_objid_intern(CTX(ctx), (const char*)bytes, (const int64_t*)offs, n, (int64_t*)keys);
  (*env)->ReleaseLongArrayElements(env, jkeys, keys, st ? JNI_ABORT : 0);
  (*env)->ReleaseByteArrayElements(env, jbytes, bytes, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, joffs, offs, JNI_ABORT);
  throw_status(env, st, CTX(ctx));
}

JNIEXPORT jbyteArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_objidDecode(JNIEnv* env, jclass cls, jlong ctx,
    jlongArray jkeys, jint n, jlongArray joffs) {
  if (n < 0 || !need_len(env, jkeys, n, "objidDecode: keys") || !need_len(env, joffs, n + 1, "objidDecode: offs"))
    return NULL;
  jlong* keys = (*env)->GetLongArrayElements(env, jkeys, NULL);
  jlong* offs = (*env)->GetLongArrayElements(env, joffs, NULL);
  int64_t cap = 32 * (int64_t)n + 64;
  char* b = (char*)malloc((size_t)cap);
  int st = b ? shim_objid_decode(CTX(ctx), (const int64_t*)keys, n, b, cap, (int64_t*)offs) : GF_ERR_NOMEM;
  if (st == GF_ERR_CAPACITY) {  /* offs[n] = the bytes needed */
    cap = offs[n];
    free(b);
    b = (char*)malloc((size_t)(cap > 0 ? cap : 1));
    st = b ? shim_objid_decode(CTX(ctx), (const int64_t*)keys, n, b, cap, (int64_t*)offs) : GF_ERR_NOMEM;
  }
  jbyteArray out = NULL;
  if (!st) {
    out = (*env)->NewByteArray(env, (jsize)offs[n]);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)offs[n], (const jbyte*)b);
  }
  free(b);
  (*env)->ReleaseLongArrayElements(env, joffs, offs, st ? JNI_ABORT : 0);
  (*env)->ReleaseLongArrayElements(env, jkeys, keys, JNI_ABORT);
  throw_status(env, st, CTX(ctx));
  return out;
}

/* ---- pinned direct buffers: a window's objID column read in place by the kernels --------- */
JNIEXPORT jobject JNICALL Java_GeoFlink_native_1_GeoFlinkHip_pinnedBuffer(JNIEnv* env, jclass cls, jlong bytes) {
  void* p = NULL;
  const int st = shim_pinned_alloc(bytes, &p);
  if (st) {
    throw_status(env, st, NULL);
    return NULL;
  }
  return (*env)->NewDirectByteBuffer(env, p, bytes);
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_pinnedFree(JNIEnv* env, jclass cls, jobject buf) {
  void* p = buf ? (*env)->GetDirectBufferAddress(env, buf) : NULL;
  if (p) shim_pinned_free(p);
}

/* ---- kNN (PointPointKNNQuery.java:132-201 + KNNQuery.java:213-272; PointPolygonKNNQuery
 * .java:245-317) ----------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnPlan(JNIEnv* env, jclass cls, jlong ctx,
    jdoubleArray jg, jdouble qx, jdouble qy, jdouble r, jint k) {
  gf_grid g;
  shim_knn* h = NULL;
  if (grid_of(env, jg, &g)) return 0;
  throw_status(env, shim_knn_plan(CTX(ctx), &g, qx, qy, r, k, &h), CTX(ctx));
  return (jlong)(intptr_t)h;
}

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnPolygonPlan(JNIEnv* env, jclass cls, jlong ctx,
    jdoubleArray jg, jintArray jro, jintArray jvo, jdoubleArray jvx, jdoubleArray jvy, jdouble r, jint k,
    jboolean approximate) {
  gf_grid g;
  shim_knn* h = NULL;
  jpolys p = {jro, jvo, jvx, jvy};
  if (grid_of(env, jg, &g) || polys_get(env, &p)) {
    polys_release(env, &p);
    return 0;
  }
  int st = shim_knn_polygon_plan(CTX(ctx), &g, &p.P, r, k, approximate, &h);
  polys_release(env, &p);
  throw_status(env, st, CTX(ctx));
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnPlanDestroy(JNIEnv* env, jclass cls, jlong plan) {
  shim_knn_destroy((shim_knn*)(intptr_t)plan);
}

/* x, y (double), objID keys (long) of one window in direct buffers; out* hold >= k entries */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnWindow(JNIEnv* env, jclass cls, jlong ctx, jlong plan,
    jobject bx, jobject by, jobject bo, jint n, jlongArray oo, jdoubleArray od, jlongArray oi, jint k) {
  const double* x = direct(env, bx, 8 * (int64_t)n, "knnWindow: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "knnWindow: y");
  const int64_t* o = direct(env, bo, 8 * (int64_t)n, "knnWindow: objID");
  (void)k;  /* the arrays are checked against the plan's own k */
  if ((*env)->ExceptionCheck(env) || !need_knn_out(env, (shim_knn*)(intptr_t)plan, oo, od, oi, "knnWindow: out"))
    return 0;
  int32_t m = 0;
  jlong* po = (*env)->GetPrimitiveArrayCritical(env, oo, NULL);
  jdouble* pd = po ? (*env)->GetPrimitiveArrayCritical(env, od, NULL) : NULL;
  jlong* pi = pd ? (*env)->GetPrimitiveArrayCritical(env, oi, NULL) : NULL;
  int st = pi ? shim_knn_window((shim_knn*)(intptr_t)plan, x, y, o, n, (int64_t*)po, pd, (int64_t*)pi, &m) : GF_ERR_NOMEM;
  if (pi) (*env)->ReleasePrimitiveArrayCritical(env, oi, pi, 0);
  if (pd) (*env)->ReleasePrimitiveArrayCritical(env, od, pd, 0);
  if (po) (*env)->ReleasePrimitiveArrayCritical(env, oo, po, 0);
  if (!pinned_ok(env, po, pd, pi)) return 0;
  throw_status(env, st, CTX(ctx));
  return m;
}

/* ---- multi-GPU kNN: RCCL exchange of the bands' records (PointPointKNNQuery.java:198-200,
 * KNNQuery.java:213-272) ------------------------------------------------------------------------ */
JNIEXPORT jbyteArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_commUniqueId(JNIEnv* env, jclass cls) {
  uint8_t id[GF_COMM_ID_BYTES];
  if (throw_status(env, shim_comm_unique_id(id), NULL)) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, GF_COMM_ID_BYTES);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, GF_COMM_ID_BYTES, (const jbyte*)id);
  return out;
}

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_commCreate(JNIEnv* env, jclass cls, jlong ctx,
    jbyteArray jid, jint nranks, jint rank) {
  if (!need_len(env, jid, GF_COMM_ID_BYTES, "commCreate: id")) return 0;
  uint8_t id[GF_COMM_ID_BYTES];
  (*env)->GetByteArrayRegion(env, jid, 0, GF_COMM_ID_BYTES, (jbyte*)id);
  shim_comm* h = NULL;
  throw_status(env, shim_comm_create(CTX(ctx), id, nranks, rank, &h), CTX(ctx));
  return (jlong)(intptr_t)h;
}

JNIEXPORT jlongArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_commCreateAll(JNIEnv* env, jclass cls,
    jintArray jdev) {
  const jsize n = jdev ? (*env)->GetArrayLength(env, jdev) : 0;
  if (n < 1 || n > 64) {
    throw_msg(env, "java/lang/IllegalArgumentException", "commCreateAll: 1..64 devices");
    return NULL;
  }
  jint dev[64];
  shim_comm* cs[64];
  (*env)->GetIntArrayRegion(env, jdev, 0, n, dev);
  if (throw_status(env, shim_comm_create_all(n, (const int*)dev, cs), NULL)) return NULL;
  jlong hs[64];
  for (jsize i = 0; i < n; ++i) hs[i] = (jlong)(intptr_t)cs[i];
  jlongArray out = (*env)->NewLongArray(env, n);
  if (out) (*env)->SetLongArrayRegion(env, out, 0, n, hs);
  return out;
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_commDestroy(JNIEnv* env, jclass cls, jlong comm) {
  shim_comm_destroy((shim_comm*)(intptr_t)comm);
}

/* this subtask's band of the window; out* hold >= k entries: the WHOLE window's neighbours */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnWindowSharded(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jlong comm, jobject bx, jobject by, jobject bo, jint n, jlong indexBase, jlongArray oo,
    jdoubleArray od, jlongArray oi, jint k) {
  const double* x = direct(env, bx, 8 * (int64_t)n, "knnWindowSharded: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "knnWindowSharded: y");
  const int64_t* o = direct(env, bo, 8 * (int64_t)n, "knnWindowSharded: objID");
  (void)k;  /* the arrays are checked against the plan's own k */
  if ((*env)->ExceptionCheck(env) || !need_knn_out(env, (shim_knn*)(intptr_t)plan, oo, od, oi, "knnWindowSharded: out"))
    return 0;
  /* not GetPrimitiveArrayCritical: the call blocks on a collective with the other ranks */
  int32_t m = 0;
  jlong* po = (*env)->GetLongArrayElements(env, oo, NULL);
  jdouble* pd = (*env)->GetDoubleArrayElements(env, od, NULL);
  jlong* pi = (*env)->GetLongArrayElements(env, oi, NULL);
  int st = po && pd && pi ? shim_knn_window_sharded((shim_knn*)(intptr_t)plan, (shim_comm*)(intptr_t)comm, x, y, o, n,
                                                    indexBase, (int64_t*)po, pd, (int64_t*)pi, &m)
                          : GF_ERR_NOMEM;
  if (pi) (*env)->ReleaseLongArrayElements(env, oi, pi, st ? JNI_ABORT : 0);
  if (pd) (*env)->ReleaseDoubleArrayElements(env, od, pd, st ? JNI_ABORT : 0);
  if (po) (*env)->ReleaseLongArrayElements(env, oo, po, st ? JNI_ABORT : 0);
  if (!pinned_ok(env, po, pd, pi)) return 0;
  throw_status(env, st, CTX(ctx));
  return m;
}

/* ---- the batched sharded path: enqueue per window, one String exchange per B windows ---------- */
JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnShardedBegin(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jlong comm, jint batch, jlong capBytes) {
  throw_status(env, shim_knn_sharded_begin((shim_knn*)(intptr_t)plan, (shim_comm*)(intptr_t)comm, batch, capBytes),
               CTX(ctx));
}
/* this subtask's band of the next window -> its ticket (x, y, objID are copied before returning) */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnShardedEnqueue(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jobject bx, jobject by, jobject bo, jint n, jlong indexBase) {
  const double* x = direct(env, bx, 8 * (int64_t)n, "knnShardedEnqueue: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "knnShardedEnqueue: y");
  const int64_t* o = direct(env, bo, 8 * (int64_t)n, "knnShardedEnqueue: objID");
  if ((*env)->ExceptionCheck(env)) return -1;
  int64_t t = -1;
  throw_status(env, shim_knn_sharded_enqueue((shim_knn*)(intptr_t)plan, x, y, o, n, indexBase, &t), CTX(ctx));
  return t;
}
JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnShardedFlush(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan) {
  throw_status(env, shim_knn_sharded_flush((shim_knn*)(intptr_t)plan), CTX(ctx));
}
/* a ticket's merged neighbours: outDist, outIdx (global) and owned (1 = a Point of this band);
 * returns their number; the arrays hold >= the plan's k */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnShardedResult(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jlong ticket, jdoubleArray od, jlongArray oi, jintArray ow) {
  shim_knn* h = (shim_knn*)(intptr_t)plan;
  const jsize k = (jsize)shim_knn_k(h);
  if (!need_len(env, od, k, "knnShardedResult: out") || !need_len(env, oi, k, "knnShardedResult: out") ||
      !need_len(env, ow, k, "knnShardedResult: out"))
    return 0;
  /* not GetPrimitiveArrayCritical: a flagged window's second exchange waits on the other ranks */
  int32_t m = 0;
  jdouble* pd = (*env)->GetDoubleArrayElements(env, od, NULL);
  jlong* pi = (*env)->GetLongArrayElements(env, oi, NULL);
  jint* pw = (*env)->GetIntArrayElements(env, ow, NULL);
  int st = pd && pi && pw ? shim_knn_sharded_result(h, ticket, pd, (int64_t*)pi, (int32_t*)pw, &m) : GF_ERR_NOMEM;
  if (pw) (*env)->ReleaseIntArrayElements(env, ow, pw, st ? JNI_ABORT : 0);
  if (pi) (*env)->ReleaseLongArrayElements(env, oi, pi, st ? JNI_ABORT : 0);
  if (pd) (*env)->ReleaseDoubleArrayElements(env, od, pd, st ? JNI_ABORT : 0);
  if (!pinned_ok(env, pd, pi, pw)) return 0;
  throw_status(env, st, CTX(ctx));
  return m;
}

/* ---- sliding kNN: the pane engine (PointPointKNNQuery.java:158,198-200) ------------------- */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnSlidingCreate(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jlong size_ms, jlong slide_ms) {
  shim_sliding* s = NULL;
  throw_status(env, shim_sliding_create((shim_knn*)(intptr_t)plan, size_ms, slide_ms, &s), CTX(ctx));
  return (jlong)(intptr_t)s;
}
JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnSlidingDestroy(JNIEnv* env, jclass cls, jlong s) {
  shim_sliding_destroy((shim_sliding*)(intptr_t)s);
}
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnSlidingPaneMs(JNIEnv* env, jclass cls, jlong s) {
  int64_t p = 0;
  shim_sliding_pane_ms((shim_sliding*)(intptr_t)s, &p);
  return p;
}
/* returns the end (ms) of the window the pane closed, or -1 */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnSlidingPush(JNIEnv* env, jclass cls, jlong ctx,
    jlong s, jlong pane, jobject bx, jobject by, jobject bo, jint n) {
  const double* x = direct(env, bx, 8 * (int64_t)n, "knnSlidingPush: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "knnSlidingPush: y");
  const int64_t* o = direct(env, bo, 8 * (int64_t)n, "knnSlidingPush: objID");
  if ((*env)->ExceptionCheck(env)) return -1;
  int32_t closed = 0;
  int64_t end = -1;
  int st = shim_sliding_push((shim_sliding*)(intptr_t)s, pane, x, y, o, n, &closed, &end);
  throw_status(env, st, CTX(ctx));
  return !st && closed ? end : -1;
}
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_knnSlidingDecode(JNIEnv* env, jclass cls, jlong ctx,
    jlong s, jlong window_end, jlongArray oo, jdoubleArray od, jlongArray oi, jint k) {
  (void)k;  /* the arrays are checked against the plan's own k */
  if (!need_knn_out(env, shim_sliding_plan((shim_sliding*)(intptr_t)s), oo, od, oi, "knnSlidingDecode: out")) return 0;
  int32_t m = 0;
  jlong* po = (*env)->GetPrimitiveArrayCritical(env, oo, NULL);
  jdouble* pd = po ? (*env)->GetPrimitiveArrayCritical(env, od, NULL) : NULL;
  jlong* pi = pd ? (*env)->GetPrimitiveArrayCritical(env, oi, NULL) : NULL;
  int st = pi ? shim_sliding_decode((shim_sliding*)(intptr_t)s, window_end, (int64_t*)po, pd, (int64_t*)pi, &m)
              : GF_ERR_NOMEM;
  if (pi) (*env)->ReleasePrimitiveArrayCritical(env, oi, pi, 0);
  if (pd) (*env)->ReleasePrimitiveArrayCritical(env, od, pd, 0);
  if (po) (*env)->ReleasePrimitiveArrayCritical(env, oo, po, 0);
  if (!pinned_ok(env, po, pd, pi)) return 0;
  throw_status(env, st, CTX(ctx));
  return m;
}

/* ---- range (PointPointRangeQuery.java:150-186, PointPolygonRangeQuery.java:170-204) -------- */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangePlan(JNIEnv* env, jclass cls, jlong ctx,
    jdoubleArray jg, jdoubleArray jqx, jdoubleArray jqy, jdouble r, jboolean approximate) {
  gf_grid g;
  shim_range* h = NULL;
  if (grid_of(env, jg, &g)) return 0;
  const jsize nq = jqx ? (*env)->GetArrayLength(env, jqx) : -1;
  if (nq < 0 || !need_len(env, jqy, nq, "rangePlan: qy")) return 0;
  jdouble* qx = (*env)->GetDoubleArrayElements(env, jqx, NULL);
  jdouble* qy = (*env)->GetDoubleArrayElements(env, jqy, NULL);
  int st = shim_range_plan(CTX(ctx), &g, qx, qy, nq, r, approximate, &h);
  (*env)->ReleaseDoubleArrayElements(env, jqy, qy, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, jqx, qx, JNI_ABORT);
  throw_status(env, st, CTX(ctx));
  return (jlong)(intptr_t)h;
}

JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangePolygonPlan(JNIEnv* env, jclass cls, jlong ctx,
    jdoubleArray jg, jintArray jro, jintArray jvo, jdoubleArray jvx, jdoubleArray jvy, jdouble r,
    jboolean approximate) {
  gf_grid g;
  shim_range* h = NULL;
  jpolys p = {jro, jvo, jvx, jvy};
  if (grid_of(env, jg, &g) || polys_get(env, &p)) {
    polys_release(env, &p);
    return 0;
  }
  int st = shim_range_polygon_plan(CTX(ctx), &g, &p.P, r, approximate, &h);
  polys_release(env, &p);
  throw_status(env, st, CTX(ctx));
  return (jlong)(intptr_t)h;
}

JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangePlanDestroy(JNIEnv* env, jclass cls, jlong plan) {
  shim_range_destroy((shim_range*)(intptr_t)plan);
}

/* emitted point indices, ascending, into the direct int buffer out (capacity outCap ints);
 * returns their count -- larger than outCap: the buffer was too small, call again with more */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeWindow(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jobject bx, jobject by, jint n, jobject bout, jint out_cap) {
  const double* x = direct(env, bx, 8 * (int64_t)n, "rangeWindow: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "rangeWindow: y");
  int32_t* out = direct(env, bout, 4 * (int64_t)out_cap, "rangeWindow: out");
  if ((*env)->ExceptionCheck(env)) return 0;
  int64_t count = 0;
  int st = shim_range_window((shim_range*)(intptr_t)plan, x, y, n, out, out_cap, &count);
  if (st != GF_ERR_CAPACITY) throw_status(env, st, CTX(ctx));
  return count;
}

/* approximate point-point range with |Q| > 1: the points of the last rangeWindow the reference
 * emits once per query point (PointPointRangeQuery.java:158-161); returns their count (> outCap:
 * call again with a larger buffer), 0 for other plans */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeWindowMulti(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jobject bout, jint out_cap) {
  int32_t* out = direct(env, bout, 4 * (int64_t)out_cap, "rangeWindowMulti: out");
  if ((*env)->ExceptionCheck(env)) return 0;
  int64_t count = 0;
  int st = shim_range_window_multi((shim_range*)(intptr_t)plan, out, out_cap, &count);
  if (st != GF_ERR_CAPACITY) throw_status(env, st, CTX(ctx));
  return count;
}

/* ---- sliding range: the pane engine (PointPointRangeQuery.java:149-186) -------------------- */
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeSlidingCreate(JNIEnv* env, jclass cls, jlong ctx,
    jlong plan, jlong size_ms, jlong slide_ms) {
  shim_range_sliding* s = NULL;
  throw_status(env, shim_range_sliding_create((shim_range*)(intptr_t)plan, size_ms, slide_ms, &s), CTX(ctx));
  return (jlong)(intptr_t)s;
}
JNIEXPORT void JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeSlidingDestroy(JNIEnv* env, jclass cls, jlong s) {
  shim_range_sliding_destroy((shim_range_sliding*)(intptr_t)s);
}
JNIEXPORT jlong JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeSlidingPaneMs(JNIEnv* env, jclass cls, jlong s) {
  int64_t p = 0;
  shim_range_sliding_pane_ms((shim_range_sliding*)(intptr_t)s, &p);
  return p;
}
/* the closed window's emitted points (window-local, ascending) with windowEnd[0] = its end, or
 * null when the pane closed no window holding a point */
JNIEXPORT jintArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_rangeSlidingPush(JNIEnv* env, jclass cls, jlong ctx,
    jlong s, jlong pane, jobject bx, jobject by, jint n, jlongArray jend) {
  const double* x = direct(env, bx, 8 * (int64_t)n, "rangeSlidingPush: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "rangeSlidingPush: y");
  if ((*env)->ExceptionCheck(env) || !need_len(env, jend, 1, "rangeSlidingPush: windowEnd")) return NULL;
  int64_t end = -1, count = 0;
  const uint32_t* idx = NULL;
  int st = shim_range_sliding_push((shim_range_sliding*)(intptr_t)s, pane, x, y, n, &end, &idx, &count);
  if (throw_status(env, st, CTX(ctx)) || end < 0) return NULL;
  jlong e = end;
  (*env)->SetLongArrayRegion(env, jend, 0, 1, &e);
  jintArray out = (*env)->NewIntArray(env, (jsize)count);
  if (out && count) (*env)->SetIntArrayRegion(env, out, 0, (jsize)count, (const jint*)idx);
  return out;
}

/* ---- joins (JoinQuery.java:73-115, PointPointJoinQuery.java:148-182,
 * PointPolygonJoinQuery.java:154-213) -> long[2m] of (ordinary / point, query / polygon) ------ */
static jlongArray pairs_array(JNIEnv* env, const uint32_t* pairs, int64_t m) {
  jlongArray out = (*env)->NewLongArray(env, (jsize)(2 * m));
  if (!out) return NULL;
  jlong* po = (*env)->GetPrimitiveArrayCritical(env, out, NULL);
  for (int64_t i = 0; i < 2 * m; ++i) po[i] = pairs[i];
  (*env)->ReleasePrimitiveArrayCritical(env, out, po, 0);
  return out;
}

JNIEXPORT jlongArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_joinWindow(JNIEnv* env, jclass cls, jlong ctx,
    jdoubleArray jug, jdoubleArray jqg, jobject box, jobject boy, jint no, jobject bqx, jobject bqy, jint nq,
    jdouble r, jboolean approximate) {
  gf_grid ug, qg;
  if (grid_of(env, jug, &ug) || grid_of(env, jqg, &qg)) return NULL;
  const double* ox = direct(env, box, 8 * (int64_t)no, "joinWindow: ox");
  const double* oy = direct(env, boy, 8 * (int64_t)no, "joinWindow: oy");
  const double* qx = direct(env, bqx, 8 * (int64_t)nq, "joinWindow: qx");
  const double* qy = direct(env, bqy, 8 * (int64_t)nq, "joinWindow: qy");
  if ((*env)->ExceptionCheck(env)) return NULL;
  const uint32_t* pairs = NULL;
  int64_t m = 0;
  int st = shim_join_window(CTX(ctx), &ug, &qg, ox, oy, no, qx, qy, nq, r, approximate, &pairs, &m);
  if (throw_status(env, st, CTX(ctx))) return NULL;
  return pairs_array(env, pairs, m);
}

JNIEXPORT jlongArray JNICALL Java_GeoFlink_native_1_GeoFlinkHip_polygonJoinWindow(JNIEnv* env, jclass cls,
    jlong ctx, jdoubleArray jg, jobject bx, jobject by, jint n, jintArray jro, jintArray jvo, jdoubleArray jvx,
    jdoubleArray jvy, jdouble r, jboolean approximate) {
  gf_grid g;
  if (grid_of(env, jg, &g)) return NULL;
  const double* x = direct(env, bx, 8 * (int64_t)n, "polygonJoinWindow: x");
  const double* y = direct(env, by, 8 * (int64_t)n, "polygonJoinWindow: y");
  if ((*env)->ExceptionCheck(env)) return NULL;
  jpolys p = {jro, jvo, jvx, jvy};
  const uint32_t* pairs = NULL;
  int64_t m = 0;
  int st = polys_get(env, &p);
  if (!st) st = shim_polygon_join_window(CTX(ctx), &g, x, y, n, &p.P, r, approximate, &pairs, &m);
  polys_release(env, &p);
  if (throw_status(env, st, CTX(ctx))) return NULL;
  return pairs_array(env, pairs, m);
}

/* ---- ingest (Deserialization.java:149-211, 291-325) ----------------------------------------
 * a chunk of complete lines in a direct buffer -> x, y, objID keys, ts (direct buffers of
 * `capacity` entries); returns the points parsed.  A bad line throws IllegalArgumentException
 * naming its index and kind -- the reference's map would have thrown on it. */
static jint parse_out(JNIEnv* env, shim_ctx* c, int st, int64_t n, int64_t bad_line, int32_t bad_kind) {
  if (st == GF_ERR_ARG && bad_line >= 0) {
    char msg[160];
    snprintf(msg, sizeof msg, "line %lld: %s (kind %d)", (long long)bad_line,
             bad_kind == GF_CSV_NUMBER_FORMAT ? "NumberFormatException" : "malformed record", (int)bad_kind);
    throw_msg(env, bad_kind == GF_CSV_NUMBER_FORMAT ? "java/lang/NumberFormatException"
                                                   : "java/lang/IllegalArgumentException", msg);
    return 0;
  }
  if (st == GF_ERR_CAPACITY) {
    throw_msg(env, "java/lang/IndexOutOfBoundsException", "parse: more lines than capacity");
    return 0;
  }
  throw_status(env, st, c);
  return st ? 0 : (jint)n;
}

JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_csvParse(JNIEnv* env, jclass cls, jlong ctx,
    jobject btext, jint len, jchar delimiter, jintArray jschema, jobject bx, jobject by, jobject bo, jobject bt,
    jint capacity) {
  const char* text = direct(env, btext, len, "csvParse: text");
  double* x = direct(env, bx, 8 * (int64_t)capacity, "csvParse: x");
  double* y = direct(env, by, 8 * (int64_t)capacity, "csvParse: y");
  int64_t* o = direct(env, bo, 8 * (int64_t)capacity, "csvParse: objID");
  int64_t* t = direct(env, bt, 8 * (int64_t)capacity, "csvParse: ts");
  if ((*env)->ExceptionCheck(env) || !need_len(env, jschema, 4, "csvParse: schema {objID, ts, x, y}")) return 0;
  gf_csv_schema sc;
  memset(&sc, 0, sizeof sc);
  jint s[4];
  (*env)->GetIntArrayRegion(env, jschema, 0, 4, s);
  sc.delimiter = (char)delimiter;
  sc.objid_field = s[0];
  sc.time_field = s[1];
  sc.x_field = s[2];
  sc.y_field = s[3];
  int64_t n = 0, bad_line = -1;
  int32_t bad_kind = 0;
  int st = shim_csv_parse(CTX(ctx), text, len, &sc, x, y, o, t, capacity, &n, &bad_line, &bad_kind);
  return parse_out(env, CTX(ctx), st, n, bad_line, bad_kind);
}

/* GeoJSONToTSpatial(uGrid, dateFormat, propertyTimeStamp, propertyObjID) (Deserialization.java:
 * 64-70,158-165): dateFormat null -> 0 (integer ms), else 1 ("yyyy-MM-dd HH:mm:ss", the only
 * pattern restated; another throws IllegalArgumentException); tzOffsetMinutes =
 * TimeZone.getDefault().getRawOffset() / 60000 on the Java side; valueLines = each line is the
 * record's value (Serialization.PointToGeoJSONOutputSchema output) instead of the Kafka record */
JNIEXPORT jint JNICALL Java_GeoFlink_native_1_GeoFlinkHip_geoJsonParse(JNIEnv* env, jclass cls, jlong ctx,
    jobject btext, jint len, jstring jts_prop, jstring jobj_prop, jstring jdate_format, jint tz_offset_minutes,
    jboolean value_lines, jobject bx, jobject by, jobject bo, jobject bt, jint capacity) {
  const char* text = direct(env, btext, len, "geoJsonParse: text");
  double* x = direct(env, bx, 8 * (int64_t)capacity, "geoJsonParse: x");
  double* y = direct(env, by, 8 * (int64_t)capacity, "geoJsonParse: y");
  int64_t* o = direct(env, bo, 8 * (int64_t)capacity, "geoJsonParse: objID");
  int64_t* t = direct(env, bt, 8 * (int64_t)capacity, "geoJsonParse: ts");
  if ((*env)->ExceptionCheck(env)) return 0;
  gf_geojson_schema sc;
  memset(&sc, 0, sizeof sc);
  const char* fmt = jdate_format ? (*env)->GetStringUTFChars(env, jdate_format, NULL) : NULL;
  if (fmt && strcmp(fmt, "yyyy-MM-dd HH:mm:ss") != 0) {
    (*env)->ReleaseStringUTFChars(env, jdate_format, fmt);
    throw_msg(env, "java/lang/IllegalArgumentException", "geoJsonParse: dateFormat other than yyyy-MM-dd HH:mm:ss");
    return 0;
  }
  sc.date_format = fmt ? 1 : 0;
  sc.tz_offset_minutes = tz_offset_minutes;
  sc.value_lines = value_lines ? 1 : 0;
  sc.time_property = jts_prop ? (*env)->GetStringUTFChars(env, jts_prop, NULL) : NULL;
  sc.objid_property = jobj_prop ? (*env)->GetStringUTFChars(env, jobj_prop, NULL) : NULL;
  int64_t n = 0, bad_line = -1;
  int32_t bad_kind = 0;
  int st = shim_geojson_parse(CTX(ctx), text, len, &sc, x, y, o, t, capacity, &n, &bad_line, &bad_kind);
  if (sc.objid_property) (*env)->ReleaseStringUTFChars(env, jobj_prop, sc.objid_property);
  if (sc.time_property) (*env)->ReleaseStringUTFChars(env, jts_prop, sc.time_property);
  if (fmt) (*env)->ReleaseStringUTFChars(env, jdate_format, fmt);
  return parse_out(env, CTX(ctx), st, n, bad_line, bad_kind);
}
